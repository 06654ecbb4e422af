import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import goldens, gpu_harness as gh
from oracle import dad_oracle
name, s = sys.argv[1], int(sys.argv[2])
d, spec, cfg = goldens.load(name)
step = gh.make_step(cfg, anchors=d["anchors"])
orc = dad_oracle.DADOracle(*goldens.problem(spec), cfg, anchors=d["anchors"])
st = goldens.state(spec, s)
gh.load_state(step, st); orc.load_state(st)
inp = goldens.step_inputs(spec, s)
epoch = int(d["s%d_epoch" % s]); lr = float(d["s%d_lr" % s])
o = gh.run_step(step, inp, epoch, lr=lr)
r = orc.step(inp, epoch, lr=lr)
B, T = spec["B"], spec["T"]
ge = gh.ws_ge(step, B, T, B, T)
for nm, a, b in (("ge_clean", ge[:B], r["e_clean_grad"]), ("ge_strong", ge[B:], r["e_strong_grad"]),
                 ("e_clean", o["e_clean"], r["e_clean"]), ("e_strong", o["e_strong"], r["e_strong"])):
    err = np.abs(a - b); rowmax = err.max(1); i = int(rowmax.argmax())
    print(nm, "rel %.3e" % (err.max() / np.abs(b).max()), "worst row", i, "rowerr %.3e" % rowmax[i],
          "row|max| %.3e" % np.abs(b[i]).max(), "rows>1e-5rel:", int((rowmax > 1e-5 * np.abs(b).max()).sum()))
print("mask", o["mask"].astype(int).tolist())
print("pred", o["pred"].astype(int).tolist())
print("ecda terms", o["ecda_terms"], "loss", o["ecda_loss"], r["ecda_loss"])
g0 = o["grads"][0]; r0 = r["grads"][0]
err = np.abs(g0 - r0); h, dd = np.unravel_index(err.argmax(), err.shape)
print("dW1 worst", h, dd, g0[h, dd], r0[h, dd], "row h err max %.3e" % err[h].max(), "row h |max| %.3e" % np.abs(r0[h]).max())
# which branch: recompute oracle contributions with GPU ge
x_c = inp["xc"]; 
print("db1 rel %.3e" % (np.abs(o["grads"][1] - r["grads"][1]).max() / np.abs(r["grads"][1]).max()))
