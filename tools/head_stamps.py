"""Diagnostic: dad_tail_ecda phase timeline (tail block and ECDA class blocks) (build variant 'stamps', -DDAD_PROBE_STAMPS;
never the product library).  Runs bench-shaped steps and prints the last step's phases."""
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
    model = PKG.SSRLModel().cuda()
    P = bench.init_model_weights(model, seed=0)
    step = PKG.DADStep(model, flavor="iemocap", precision="bf16", rng="counter", seed=1)
    data = bench.make_batches(P, 2, B, T, seed=17, device=torch.device("cuda"))
    for i in range(8):
        step.step(data[i % 2][0], data[i % 2][1], 60)
    torch.cuda.synchronize()
    L = PKG.lib()
    ebuf = (ctypes.c_ulonglong * (4 * 16 + 12))()
    assert L.dad_probe_read_ecda_stamps(ebuf, len(ebuf)) == 0
    e = np.frombuffer(ebuf, dtype=np.uint64).astype(np.int64)
    t0 = e[64]
    rel = lambda v: (v - t0) / 100.0
    tn = ["end", "ce", "probs", "dacp", "kl", "outputs", "clsbwd"]
    print("tail start 0 | " + "  ".join("%s %.2f" % (tn[k - 1], rel(e[64 + k])) for k in range(1, 8) if e[64 + k] > 0))
    names = ["start", "meta", "centroid", "gates", "pdist", "compact", "stage", "mmd", "grads"]
    for c in range(4):
        row = e[c * 16:c * 16 + 16]
        parts = ["%s %.2f" % (names[k], rel(row[k])) for k in range(9) if row[k] > 0]
        sub = ["%s %.2f" % (nm, rel(row[k])) for k, nm in ((12, "dist"), (13, "sumD"), (14, "coef"), (15, "terms")) if row[k] > 0]
        print("ecda class %d (n=%d ns=%d): %s | mmd: %s" % (c, e[c * 16 + 10], e[c * 16 + 11], "  ".join(parts), "  ".join(sub)))


if __name__ == "__main__":
    main()
