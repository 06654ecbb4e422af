"""Diagnostic: host-side cost of DADStep.step (Python + ctypes + HIP enqueue) vs the GPU step.

Prints per-step host time of each phase (prepare, the three ABI calls, losses()) and the wall
time per step with and without per-step synchronisation."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

PKG = bench.PKG


def main():
    B, T, N = 64, 300, 200
    dev = torch.device("cuda")
    model = PKG.SSRLModel().to(dev)
    P = bench.init_model_weights(model, seed=0)
    step = PKG.DADStep(model, flavor="iemocap", precision="bf16", rng="counter", seed=1)
    data = bench.make_batches(P, 4, B, T, seed=17, device=dev)
    for i in range(10):
        step.step(data[i % 4][0], data[i % 4][1], 60)
    torch.cuda.synchronize()
    acc = {}
    L = PKG.lib()

    def wrap(obj, name, key):
        f = getattr(obj, name)

        def w(*a, **k):
            t0 = time.perf_counter()
            r = f(*a, **k)
            acc[key] = acc.get(key, 0.0) + time.perf_counter() - t0
            return r
        setattr(obj, name, w)

    wrap(step, "_prepare", "prepare")
    wrap(step, "_workspace", "workspace")
    wrap(step, "losses", "losses")
    for n in ("dad_step_encode", "dad_step_backward", "dad_step_apply"):
        wrap(L, n, n)
    t0 = time.perf_counter()
    for i in range(N):
        step.step(data[i % 4][0], data[i % 4][1], 60)
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_wall = time.perf_counter() - t0
    print("host dispatch %.1f us/step, wall %.1f us/step" % (t_host / N * 1e6, t_wall / N * 1e6))
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
        print("  %-20s %7.1f us/step" % (k, v / N * 1e6))
    t0 = time.perf_counter()
    for i in range(50):
        step.step(data[i % 4][0], data[i % 4][1], 60)
        torch.cuda.synchronize()
    print("synchronised step %.1f us" % ((time.perf_counter() - t0) / 50 * 1e6))


if __name__ == "__main__":
    main()
