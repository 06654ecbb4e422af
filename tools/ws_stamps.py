"""Diagnostic: per-workgroup timeline of dad_encode_ws (build variant 'stamps', compiled with
-DDAD_PROBE_STAMPS; never the product library).  Runs bench-shaped steps, then reads the
wave-0 stamps of every workgroup of the last launch and summarises them per role."""
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
    step = PKG.DADStep(model, flavor="iemocap", precision=os.environ.get("STAMP_PREC", "fp16"), rng="counter", seed=1)
    data = bench.make_batches(P, 2, B, T, seed=17, device=torch.device("cuda"))
    for i in range(8):
        step.step(data[i % 2][0], data[i % 2][1], 60)
    torch.cuda.synchronize()
    L = PKG.lib()
    n = 256
    buf = (ctypes.c_ulonglong * (10 * n))()
    assert L.dad_probe_read_ws_stamps(buf, 10 * n) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(n, 10).astype(np.int64)
    st = st[st[:, 0] > 0]
    t0 = st[:, 0].min()
    start, pro, end = (st[:, 0] - t0) / 100.0, (st[:, 1] - t0) / 100.0, (st[:, 2] - t0) / 100.0
    role = st[:, 3] >> 16
    Q = st[:, 3] & 0xffff
    for r, name in ((1, "teacher"), (0, "student")):
        m = role == r
        if not m.any():
            continue
        per = (end[m] - pro[m]) / Q[m]
        print("%-7s n=%3d Q p50 %d  start p50/max %.1f/%.1f  prologue-end p50 %.1f  end p50/max %.1f/%.1f us  "
              "loop us/sub-slab p50 %.3f" % (name, m.sum(), np.median(Q[m]), np.median(start[m]), start[m].max(),
                                            np.median(pro[m]), np.median(end[m]), end[m].max(), np.median(per)))
        cyc = st[m, 4:10].astype(np.float64) / Q[m][:, None]
        if r == 0:
            kinds = student_kinds(64, 300, int((role == 1).sum()), int(m.sum()))
            loop = (end[m] - pro[m])
            A = kinds.astype(np.float64)
            coef, *_ = np.linalg.lstsq(A, loop, rcond=None)
            print("        fit: clean sub-slab %.3f us, strong sub-slab %.3f us" % tuple(coef))
        print("        wave-0 cycles/sub-slab p50: wait %.0f  mfma %.0f  convert %.0f  epilogue %.0f  dma %.0f  barrier %.0f" %
              tuple(np.median(cyc, axis=0)))
        if r == 0:
            # per-kind phase cycles: least squares of each workgroup's phase sums on its sub-slab counts
            sums = st[m, 4:10].astype(np.float64)
            fit, *_ = np.linalg.lstsq(A, sums, rcond=None)
            for kname, row in (("clean", fit[0]), ("strong", fit[1])):
                print("        %-6s fit cycles/sub-slab: wait %.0f  mfma %.0f  convert %.0f  epilogue %.0f  dma %.0f  barrier %.0f"
                      % ((kname,) + tuple(row)))


def student_kinds(B, T, nt, ns, wstrong=1.47):
    """(clean, strong) sub-slab counts of each student workgroup (mirror of job_range)."""
    nc = (T + 31) // 32
    Jc = Js = B * nc
    wtot = Jc + Js * wstrong
    def at(k):
        if k >= ns:
            return Jc + Js
        b = np.float32(wtot) * np.float32(k) / np.float32(ns)
        j = int(b + 0.5) if b <= Jc else Jc + int((b - Jc) / wstrong + 0.5)
        return min(max(j, 0), Jc + Js)
    out = []
    for k in range(ns):
        j0, j1 = at(k), at(k + 1)
        clean = max(0, min(j1, Jc) - j0)
        out.append((2 * clean, 2 * (j1 - j0 - clean)))
    return np.array(out)


if __name__ == "__main__":
    main()
