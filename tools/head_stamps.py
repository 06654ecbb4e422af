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
    step = PKG.DADStep(model, flavor="iemocap", precision=os.environ.get("STAMP_PREC", "fp16"), rng="counter", seed=1)
    data = bench.make_batches(P, 2, B, T, seed=17, device=torch.device("cuda"))
    S = 32  # slots per ECDA class (tail.hip ECDA_SLOTS)
    L = PKG.lib()
    reps = int(os.environ.get("STAMP_REPS", "15"))
    raw = []
    for r in range(reps):   # the last step of a 4-step burst, reps times
        for i in range(4):
            # STAMP_AHEAD=1: each step names the next batch (the bench's shape: the tail launch also
            # prepares the next batch's noisy rows)
            nxt = data[(i + 1) % 2] if os.environ.get("STAMP_AHEAD") == "1" else None
            step.step(data[i % 2][0], data[i % 2][1], 60, next_batch=nxt)
        torch.cuda.synchronize()
        ebuf = (ctypes.c_ulonglong * (4 * S + 16))()
        assert L.dad_probe_read_ecda_stamps(ebuf, len(ebuf)) == 0
        raw.append(np.frombuffer(ebuf, dtype=np.uint64).astype(np.int64))
    raw = np.stack(raw[2:] if reps > 4 else raw)
    t0 = raw[:, 4 * S:4 * S + 1]
    relm = np.median((raw - t0) / 100.0, axis=0)        # us after the tail block's start, median
    setm = np.all(raw > 0, axis=0)
    last = raw[-1]
    on = lambda k: bool(setm[k])
    rel = lambda k: relm[k]
    T = 4 * S
    tn = ["end", "ce", "probs", "dacp", "kl", "outputs", "clsbwd"]
    print("median of %d steps" % raw.shape[0])
    if on(T + 14):
        ends = [rel(c * S + 8) for c in range(4) if on(c * S + 8)]
        print("launch entry %.2f (tail start 0 = after the pooling wait) | ECDA last class end %.2f | "
              "last preparation block end %s us" % (rel(T + 14), max(ends) if ends else float("nan"),
                                                    ("%.2f" % rel(T + 15)) if on(T + 15) else "-"))
    print("tail start 0 | " + "  ".join("%s %.2f" % (tn[k - 1], rel(T + k)) for k in range(1, 8) if on(T + k)))
    if on(T + 13) and on(T + 12):
        ghz = np.median((raw[:, T + 13] - raw[:, T + 12]) / ((raw[:, T + 1] - raw[:, T]) * 10.0))
        print("  tail block clock: %.2f GHz" % ghz)
    dn = ["dacp-ranks", "dacp-thresholds", "mask", "epoch-sums"]
    print("  tail dacp detail: " + "  ".join("%s %.2f" % (dn[k - 8], rel(T + k)) for k in range(8, 12) if on(T + k)))
    names = ["start", "meta", "centroid", "gates", "pdist", "compact", "stage", "mmd", "grads"]
    for c in range(4):
        o = c * S
        parts = ["%s %.2f" % (names[k], rel(o + k)) for k in range(9) if on(o + k)]
        sub = ["%s %.2f" % (nm, rel(o + k)) for k, nm in ((12, "dist"), (13, "sumD"), (14, "coef"), (15, "terms"),
                                                          (16, "cnt"), (17, "cpart"), (18, "cbar"), (19, "stage0"),
                                                          (20, "d-tri"), (21, "d-acc"), (22, "d-rs"))
               if on(o + k)]
        print("ecda class %d (n=%d ns=%d): %s | sub: %s" % (c, last[o + 10], last[o + 11], "  ".join(parts), "  ".join(sub)))


if __name__ == "__main__":
    main()
