"""Diagnostic: dad_tail_ecda class-block sizes and phase ends along a bench-shaped run from
initialisation (build variant 'stamps'): the ECDA cost of the driver's short run (steps 5..25)
vs the steady state.  Prints one line per class at the listed steps."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("DAD_LIB_VARIANT", "stamps")
import bench  # noqa: E402

PKG = bench.PKG


def main():
    B, T = 64, 300
    dev = torch.device("cuda")
    model = PKG.SSRLModel().to(dev)
    P = bench.init_model_weights(model, seed=0)
    import argparse
    view = bench.flavor_view(argparse.Namespace(flavor="iemocap", force_ecda=False))
    step = PKG.DADStep(model, view, precision="bf16", rng="counter", seed=1000, comm=None)
    data = bench.make_batches(P, bench.N_BATCHES, B, T, seed=17, device=dev)
    S = 24
    L = PKG.lib()
    show = [int(x) for x in os.environ.get("STEPS", "1 3 6 10 15 20 25 40 80 150 250").split()]
    names = ["start", "meta", "centroid", "gates", "pdist", "compact", "stage", "mmd", "grads"]
    for i in range(max(show) + 1):
        c, nb = data[i % len(data)]
        step.step(c, nb, 60)
        if i in show:
            torch.cuda.synchronize()
            ebuf = (ctypes.c_ulonglong * (4 * S + 16))()
            assert L.dad_probe_read_ecda_stamps(ebuf, len(ebuf)) == 0
            raw = np.frombuffer(ebuf, dtype=np.uint64).astype(np.int64)
            t0 = raw[4 * S]
            msum = float(step.outputs(B, B)["msum"])
            line = []
            for cl in range(4):
                o = cl * S
                end = max((raw[o + k] - t0) / 100.0 for k in range(9) if raw[o + k] > 0)
                line.append("c%d n=%d ns=%d end %.1f" % (cl, raw[o + 10], raw[o + 11], end))
            print("step %3d msum %2d | %s" % (i, msum, " | ".join(line)), flush=True)


if __name__ == "__main__":
    main()
