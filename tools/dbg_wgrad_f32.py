"""Debug: the fp32 step's dW1 on the first golden against the oracle, per row/column block."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import goldens  # noqa: E402
import gpu_harness as gh  # noqa: E402
from oracle import dad_oracle  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else goldens.variants()[0]
d, spec, cfg = goldens.load(name)
step = gh.make_step(cfg, anchors=d["anchors"])
orc = dad_oracle.DADOracle(*goldens.problem(spec), cfg, anchors=d["anchors"])
for s, epoch in list(goldens.schedule(d))[:2]:
    p = "s%d_" % s
    st = goldens.state(spec, s)
    gh.load_state(step, st)
    orc.load_state(st)
    inp = goldens.step_inputs(spec, s)
    lr = float(d[p + "lr"])
    o = gh.run_step(step, inp, epoch, lr=lr)
    r = orc.step(inp, epoch, lr=lr)
    g = np.asarray(o["grads"][0], np.float64)
    ref = np.asarray(r["grads"][0], np.float64) if "grads" in r else None
    print(name, "step", s, "epoch", epoch, "clip_norm", o["clip_norm"], "shape", g.shape,
          "finite", np.isfinite(g).all(), "max", np.abs(g).max())
    if ref is not None:
        err = np.abs(g - ref)
        print("  ref max", np.abs(ref).max(), "err max", err.max())
        hb = err.reshape(8, 32, 6, 128).max(axis=(1, 3))
        print("  err by (h block of 32, d block of 128):")
        print(np.array2string(hb, precision=2, max_line_width=200))
        rows = np.argwhere(err > 1e-3 * np.abs(ref).max())
        print("  bad count", len(rows), "first", rows[:10].tolist())
