"""Per-kernel times of the fp16 step on balanced against random-label batches, each from the initial
weights (bench.side_mode, fresh DADStep), and the balanced batches again after 500 training steps:
which of data, labels or weights moves the encoder and weight gradient.   python tools/data_effect.py"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

PKG = bench.PKG


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B, T = 64, 300
    model = PKG.SSRLModel().to(dev)
    P = bench.init_model_weights(model, seed=0)
    view = PKG.ConfigView(None, flavor="iemocap")
    args = argparse.Namespace(epoch=60, no_ahead=False, kernel_steps=32)
    bal = bench.make_batches(P, bench.N_BATCHES, B, T, seed=17, device=dev)
    rnd = bench.make_batches(P, bench.N_BATCHES, B, T, seed=29, device=dev, random_labels=True)
    rnd17 = bench.make_batches(P, bench.N_BATCHES, B, T, seed=17, device=dev, random_labels=True)
    step = PKG.DADStep(model, view, precision="fp16", rng="counter", seed=1000)
    snap0 = bench.snapshot(model, step)
    kt = lambda r: {k: round(v["avg_ms"] * 1e3, 1) for k, v in r["kernels"].items() if "avg_ms" in v}
    for rep in range(2):
        for name, data in (("balanced s17", bal), ("random s29", rnd), ("random s17", rnd17)):
            bench.restore(model, step, snap0)
            r = bench.side_mode(model, view, data, B, T, args, "fp16", 200)
            print("%-13s initial weights: %.4f ms %s" % (name, r["ms_per_step"], kt(r)), flush=True)
    bench.restore(model, step, snap0)
    for i in range(500):
        c, nb = bal[i % len(bal)]
        step.step(c, nb, 60, next_batch=bal[(i + 1) % len(bal)])
    torch.cuda.synchronize()
    for name, data in (("balanced s17", bal), ("random s29", rnd)):
        r = bench.side_mode(model, view, data, B, T, args, "fp16", 200)
        print("%-13s after 500 steps: %.4f ms %s" % (name, r["ms_per_step"], kt(r)), flush=True)


if __name__ == "__main__":
    main()
