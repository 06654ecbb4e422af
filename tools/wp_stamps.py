"""Diagnostic: per-workgroup timeline of dad_encode_wp (build variant 'stamps', -DDAD_PROBE_STAMPS;
never the product library).  Runs bench-shaped steps (each naming the next batch, as the bench
does), then reads the stamps of every workgroup of the last encoder launch and summarises them per
role: start / prologue end / end (us after the first workgroup's start) and wave-0 cycles per
32-row job in the ping-pong loop's phases: MFMA, the MFMA phase's end (vmcnt wait + barrier), epilogue +
DMA issue, the overhead phase's barrier."""
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
        step.step(data[i % 2][0], data[i % 2][1], 60, next_batch=data[(i + 1) % 2])
    torch.cuda.synchronize()
    L = PKG.lib()
    n = 256
    buf = (ctypes.c_ulonglong * (10 * n + 40 * n))()
    assert L.dad_probe_read_ws_stamps(buf, 10 * n + 40 * n) == 0
    allst = np.frombuffer(buf, dtype=np.uint64).astype(np.int64)
    st = allst[:10 * n].reshape(n, 10)
    pw = allst[10 * n:].reshape(n, 8, 5)          # per wave: 4 phase sums, group | SIMD << 8
    st_all = st
    st = st[st[:, 0] > 0]
    t0 = st[:, 0].min()
    start, pro, end = (st[:, 0] - t0) / 100.0, (st[:, 1] - t0) / 100.0, (st[:, 2] - t0) / 100.0
    role = st[:, 3] >> 16
    Q = st[:, 3] & 0xffff
    for r, name in ((0, "teacher"), (1, "student")):
        m = (role == r) & (Q > 0)
        if not m.any():
            continue
        per = (end[m] - pro[m]) / Q[m]
        w1 = (st[:, 8] - t0) / 100.0
        print("%-7s n=%3d Q p50 %d  start p50/max %.1f/%.1f  prologue-end p50 %.1f  W1+2 jobs landed p50/max %.1f/%.1f  "
              "end p50/max %.1f/%.1f us  loop us/sub-slab p50 %.3f"
              % (name, m.sum(), np.median(Q[m]), np.median(start[m]), start[m].max(), np.median(pro[m]),
                 np.median(w1[m]), w1[m].max(), np.median(end[m]), end[m].max(), np.median(per)))
        ends = np.sort(end[m])
        print("        end percentiles p10/p50/p90/max %.1f/%.1f/%.1f/%.1f us" % tuple(np.percentile(ends, [10, 50, 90, 100])))
        if True:
            cyc = st[m, 4:9].astype(np.float64) / (Q[m][:, None] / 2.0)
            print("        wave-0 cycles per 32-row job p50: mfma %.0f  mfma-end wait+barrier %.0f  epilogue+dma %.0f  "
                  "overhead barrier %.0f" % tuple(np.median(cyc, axis=0))[:4])
            # every wave, by group: per-job cycles (p50 over workgroups of this role)
            sel = np.nonzero(st_all[:, 0] > 0)[0][m]
            for g in (0, 1):
                rows = []
                for wg in sel:
                    jobs = (st_all[wg, 3] & 0xffff) / 2.0
                    for w in range(8):
                        if (pw[wg, w, 4] & 0xff) == g and jobs > 0:
                            rows.append(pw[wg, w, :4] / jobs)
                if rows:
                    rows = np.array(rows, dtype=np.float64)
                    print("        group %d (%d waves) cycles per job p50: mfma %.0f  mfma-end %.0f  overhead work %.0f  "
                          "overhead barrier %.0f | mfma p90 %.0f max %.0f" % ((g, len(rows)) + tuple(np.median(rows, axis=0))
                                                                        + (np.percentile(rows[:, 0], 90), rows[:, 0].max())))
            simd = [(pw[wg, w, 4] >> 8) & 3 for wg in sel[:1] for w in range(8)]
            grp = [pw[wg, w, 4] & 0xff for wg in sel[:1] for w in range(8)]
            print("        first workgroup: SIMD per wave %s, group per wave %s" % (simd, grp))


if __name__ == "__main__":
    main()
