"""Host issue cost of the timed step loop (bench.py's eager path) on the GPU box.

For K in (20, 200): the host time to enqueue K steps (no sync), the wall time to their end, and
the GPU-side time between an event before the first and after the last step; then a cProfile
of 200 enqueues (top entries by own time) so the Python work per step is visible.
    python tools/host_issue.py [--no-ahead] [--epoch=60]
"""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

PKG = bench.PKG


def main():
    ahead = "--no-ahead" not in sys.argv
    epoch = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--epoch=")), "60"))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    PKG.lib()
    model = PKG.SSRLModel().to(dev)
    P = bench.init_model_weights(model, seed=0)
    view = PKG.ConfigView(None, flavor="iemocap")
    step = PKG.DADStep(model, view, precision="fp16", rng="counter", seed=1000, comm=None)
    data = bench.make_batches(P, bench.N_BATCHES, 64, 300, seed=17, device=dev)
    pos = [0]

    def run(n):
        for _ in range(n):
            i = pos[0]
            pos[0] += 1
            c, nb = data[i % len(data)]
            step.step(c, nb, epoch, next_batch=data[(i + 1) % len(data)] if ahead else None)

    run(30)
    torch.cuda.synchronize()
    for k in (1, 5, 20, 200, 1, 5, 20, 200):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        run(k)
        t1 = time.perf_counter()
        e1.record()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print("K=%3d  host enqueue %7.1f us/step   wall %7.1f us/step   gpu(events) %7.1f us/step" %
              (k, (t1 - t0) / k * 1e6, (t2 - t0) / k * 1e6, e0.elapsed_time(e1) / k * 1e3), flush=True)
    # the first step after an idle wait: blocking sync vs a spinning wait (event polling) before it
    def spin_sync():
        ev = torch.cuda.Event()
        ev.record()
        while not ev.query():
            pass
        torch.cuda.synchronize()

    for mode in ("block", "spin", "block", "spin"):
        for k in (1, 20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            run(3)
            if mode == "spin":
                spin_sync()
            else:
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record()
            run(k)
            t1 = time.perf_counter()
            e1.record()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            print("%-5s K=%2d  host enqueue %7.1f us/step   wall %7.1f us/step   gpu(events) %7.1f us/step" %
                  (mode, k, (t1 - t0) / k * 1e6, (t2 - t0) / k * 1e6, e0.elapsed_time(e1) / k * 1e3), flush=True)
    # bench.py's sequence before its timed region: snapshot / restore (parameter copies, state
    # load, shadow refresh), optionally the KernelTimer, then K=20 timed steps
    for mode in ("plain", "restore", "restore+timer", "plain", "restore", "restore+timer"):
        run(5)
        torch.cuda.synchronize()
        timer = None
        if mode != "plain":
            snap = bench.snapshot(model, step)
            bench.restore(model, step, snap)
            torch.cuda.synchronize()
        if mode.endswith("timer"):
            timer = PKG._lib.KernelTimer(bench.event_every(20), 21, kernels=bench.TIMED_KERNELS)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        run(20)
        e1.record()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if timer is not None:
            timer.stop()
        print("%-14s K=20  wall %7.1f us/step   gpu(events) %7.1f us/step  prepped %s" %
              (mode, (t2 - t0) / 20 * 1e6, e0.elapsed_time(e1) / 20 * 1e3, step.last_prepped), flush=True)
    pr = cProfile.Profile()
    torch.cuda.synchronize()
    pr.enable()
    run(200)
    pr.disable()
    torch.cuda.synchronize()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(s.getvalue())


if __name__ == "__main__":
    main()
