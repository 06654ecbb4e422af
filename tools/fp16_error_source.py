"""Where the FP16 step's logit error comes from, on the CPU.

For every golden fixture (tests/golden) and step, the teacher-weak, student-clean and student-strong
encoder + classifier forward is recomputed in float64 from the fixture's seeded state and inputs
(oracle/synth, the same arrays the GPU replay feeds the step) with the MFMA operands rounded to fp16
(round to nearest even, as v_cvt_pk_f16_f32) in three ways: rows only, W1 only, both.  Each logit
tensor's max-abs error over max|z| is reported against the unrounded float64 forward, i.e. the error
budget of each operand rounding with an exact accumulation.  Writes a JSON table (argv[1], default
profiles/r06_fp16_error_source.json).  Test infrastructure: imports only the oracle.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))

import goldens  # noqa: E402
from oracle import dad_oracle  # noqa: E402

F16 = np.float16


def forward(x, pad, W1, b1, W2, b2, keep=None):
    """float64 encoder (masked mean of ReLU) + classifier; keep: dropout factors or None."""
    B, T, D = x.shape
    pre = (x.reshape(B * T, D).astype(np.float64) @ W1.T.astype(np.float64)).reshape(B, T, -1) + b1
    valid = ~pad
    act = (pre > 0) & valid[..., None]
    e = np.where(act, pre, 0.0).sum(axis=1) / np.maximum(valid.sum(axis=1), 1.0)[:, None]
    d = e if keep is None else e * keep
    return e, d @ W2.T.astype(np.float64) + b2


def r16(a):
    return np.asarray(a, np.float32).astype(F16).astype(np.float64)


def rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1e-12, float(np.max(np.abs(b)))))


def main(out):
    table = {}
    worst = {}
    for name in goldens.variants():
        d, spec, cfg = goldens.load(name)
        rows = {}
        for s, epoch in goldens.schedule(d):
            st = goldens.state(spec, s)
            inp = goldens.step_inputs(spec, s)
            warm = epoch < cfg["WARMUP_EPOCHS"]
            branches = {"z_clean": ("student", inp["xc"], inp["mc"], inp["keep1"])}
            if not warm:
                xw = dad_oracle.weak_augment(inp["xn"], inp["nw"], cfg["WEAK_NOISE_STD"])
                xs = dad_oracle.strong_augment(inp["xn"], inp["ns"], inp["u"], inp["start"], cfg["STRONG_NOISE_STD"],
                                               cfg["DROPOUT_RATE"], cfg["TEMPORAL_MASK_RATIO"])
                branches["z_teacher"] = ("teacher", xw, inp["mn"], None)
                branches["z_strong"] = ("student", xs, inp["mn"], inp["keep2"])
            row = {}
            for key, (net, x, pad, keep) in branches.items():
                W1, b1, W2, b2 = [np.asarray(a, np.float64) for a in st[net]]
                p = cfg["DROPOUT_RATE"]
                kp = None if keep is None or p == 0 else np.asarray(keep, np.float64) / (1.0 - p)
                _, z = forward(np.asarray(x, np.float64), pad, W1, b1, W2, b2, kp)
                _, zx = forward(r16(x), pad, W1, b1, W2, b2, kp)
                _, zw = forward(np.asarray(x, np.float64), pad, r16(W1), b1, W2, b2, kp)
                _, zb = forward(r16(x), pad, r16(W1), b1, W2, b2, kp)
                row[key] = {"rows_fp16": rel(zx, z), "w1_fp16": rel(zw, z), "both_fp16": rel(zb, z)}
                for k, v in row[key].items():
                    if v > worst.get((key, k), (0.0,))[0]:
                        worst[(key, k)] = (v, name, "s%d" % s)
            rows["s%d" % s] = row
        table[name] = rows
        print(name, {k: {kk: "%.2e" % vv for kk, vv in v.items()} for k, v in rows[max(rows)].items()}, flush=True)
    summary = {"%s.%s" % k: {"max": v[0], "fixture": v[1], "step": v[2]} for k, v in sorted(worst.items())}
    with open(out, "w") as f:
        json.dump({"what": __doc__.strip().splitlines()[0], "worst": summary, "fixtures": table}, f, indent=1)
    for k, v in summary.items():
        print("%-26s %.3e  %s %s" % (k, v["max"], v["fixture"], v["step"]))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "..", "profiles", "r06_fp16_error_source.json"))
