"""Diagnostic: dad_wgrad_direct per-phase cycles (build variant 'stamps', -DDAD_PROBE_STAMPS;
never the product library).  Runs bench-shaped steps and prints workgroup averages."""
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
    ahead = os.environ.get("STAMP_AHEAD", "0") == "1"   # 1: each step names the next (dad_wgrad_direct*_cp)
    for i in range(6):
        nxt = (data[(i + 1) % 2][0], data[(i + 1) % 2][1]) if ahead else None
        step.step(data[i % 2][0], data[i % 2][1], 60, next_batch=nxt)
    torch.cuda.synchronize()
    L = PKG.lib()
    n = 256
    buf = (ctypes.c_ulonglong * (10 * n))()
    assert L.dad_probe_read_wgd_stamps(buf, 10 * n) == 0
    e = np.frombuffer(buf, dtype=np.uint64).astype(np.float64).reshape(n, 10)
    e = e[e[:, 8] > 0]
    m = e.mean(0)
    print("workgroups %d; cycles: prologue %.0f loop %.0f epilogue %.0f" % (len(e), m[0], m[1], m[2]))
    print("prologue: to slab loads %.0f, dL/de table %.0f, first staging %.0f, barrier %.0f" % (m[3], m[6], m[7], m[0] - m[3] - m[6] - m[7]))
    print("per round (n=%.1f): compute+stage+load %.0f barrier %.0f" % (m[8], m[4] / m[8], m[5] / m[8]))
    tot = e[:, 0] + e[:, 1] + e[:, 2]
    print("total cycles per workgroup: p50 %.0f p90 %.0f max %.0f; loop p50 %.0f max %.0f; epilogue max %.0f"
          % (np.percentile(tot, 50), np.percentile(tot, 90), tot.max(), np.percentile(e[:, 1], 50), e[:, 1].max(),
             e[:, 2].max()))


if __name__ == "__main__":
    main()
