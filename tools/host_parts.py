"""Host cost of the pieces of DADStep.step() (bench geometry, fp16, next batch named): each piece
timed over many calls, then whole steps.   python tools/host_parts.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

PKG = bench.PKG
_lib = PKG._lib


def t(label, fn, n=3000):
    fn()
    a = time.perf_counter()
    for _ in range(n):
        fn()
    print("%-28s %7.2f us" % (label, (time.perf_counter() - a) / n * 1e6), flush=True)


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    PKG.lib()
    model = PKG.SSRLModel().to(dev)
    P = bench.init_model_weights(model, seed=0)
    view = PKG.ConfigView(None, flavor="iemocap")
    step = PKG.DADStep(model, view, precision="fp16", rng="counter", seed=1000)
    data = bench.make_batches(P, 2, 64, 300, seed=17, device=dev)
    (c, nb), nxt = data[0], data[1]
    step.step(c, nb, 60, next_batch=nxt)
    torch.cuda.synchronize()
    cfg, bt, keep = step._batch_structs(c, nb, 60, None, None)
    t("param_key", step._param_key)
    t("make_config", lambda: step.make_config(64, 300, 64, 300, 60))
    t("dev_batch (clean)", lambda: PKG.step._dev_batch(c, dev))
    t("batch_structs", lambda: step._batch_structs(c, nb, 60, None, None))
    t("batch_structs like", lambda: step._batch_structs(nxt[0], nxt[1], 60, None, None, like=cfg))
    t("state_struct", lambda: step._state_struct(64, 64))
    t("torch.empty(4)", lambda: torch.empty(4, device=dev))
    t("prep_key", lambda: step._prep_key(cfg, bt))
    t("workspace", lambda: step._workspace(cfg))
    t("losses()", step.losses)
    t("stream handle", step._stream)
    torch.cuda.synchronize()
    for k in range(3):
        n = 200
        a = time.perf_counter()
        for i in range(n):
            cc, nn = data[i % 2]
            step.step(cc, nn, 60, next_batch=data[(i + 1) % 2])
        b = time.perf_counter()
        torch.cuda.synchronize()
        print("step() enqueue %7.2f us   wall %7.2f us" % ((b - a) / n * 1e6, (time.perf_counter() - a) / n * 1e6))


if __name__ == "__main__":
    main()
