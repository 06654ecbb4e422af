"""Diagnostic: per-workgroup timeline of dad_encode_bf16 (build variant 'stamps', compiled
with -DDAD_PROBE_STAMPS; never the product library).  Runs bench-shaped steps, then reads
[start, loop-end, end] wall clocks (100 MHz) per workgroup of the last launch."""
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
    for i in range(6):
        step.step(data[i % 2][0], data[i % 2][1], 60)
    torch.cuda.synchronize()
    L = PKG.lib()
    ncn = ncc = (T + 31) // 32
    n_noisy = (B * ncn + 3) // 4
    nwg = n_noisy + (B * ncc + 7) // 8
    buf = (ctypes.c_ulonglong * (3 * nwg))()
    rc = L.dad_probe_read_stamps(buf, nwg)
    assert rc == 0, rc
    st = np.frombuffer(buf, dtype=np.uint64).reshape(nwg, 3).astype(np.int64)
    t0 = st[:, 0].min()
    us = (st - t0) / 100.0            # 100 MHz -> us
    ebuf = (ctypes.c_ulonglong * (4 * 12 + 4))()
    if hasattr(L, "dad_probe_read_ecda_stamps") and L.dad_probe_read_ecda_stamps(ebuf) == 0:
        e = np.frombuffer(ebuf, dtype=np.uint64).astype(np.int64)
        rel = lambda v: (v - t0) / 100.0
        print("encoder end %.1f us; tail %.1f -> %.1f us" % (us[:, 2].max(), rel(e[48]), rel(e[49])))
        names = ["start", "meta", "centroid", "gates", "zero", "compact", "stage", "mmd", "grads"]
        for c in range(4):
            row = e[c * 12:c * 12 + 9]
            parts = ["%s %.1f" % (names[k], rel(row[k])) for k in range(9) if row[k] > 0]
            print("ecda class %d (n=%d ns=%d): %s" % (c, e[c * 12 + 10], e[c * 12 + 11], "  ".join(parts)))
    for name, sl in (("noisy", slice(0, n_noisy)), ("clean", slice(n_noisy, nwg))):
        s = us[sl]
        print("%-5s n=%3d start p0/p50/p100 %.1f/%.1f/%.1f  loop p50/p100 %.1f/%.1f  epi p50/p100 %.1f/%.1f  "
              "end p50/p100 %.1f/%.1f us" % (
                  name, len(s), s[:, 0].min(), np.median(s[:, 0]), s[:, 0].max(),
                  np.median(s[:, 1] - s[:, 0]), (s[:, 1] - s[:, 0]).max(),
                  np.median(s[:, 2] - s[:, 1]), (s[:, 2] - s[:, 1]).max(), np.median(s[:, 2]), s[:, 2].max()))


if __name__ == "__main__":
    main()
