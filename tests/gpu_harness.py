"""Drive the fused HIP step and the oracle from the same seeded state (GPU tests only)."""
import numpy as np
import torch

import dadpkg
from oracle import dad_oracle

P = 256 * 768 + 256 + 4 * 256 + 4


def flat(params):
    return np.concatenate([np.asarray(a, np.float32).reshape(-1) for a in params])


def unflat(v):
    v = np.asarray(v, np.float32)
    o = [0, 256 * 768, 256 * 768 + 256, 256 * 768 + 256 + 1024, P]
    shapes = [(256, 768), (256,), (4, 256), (4,)]
    return [v[o[i]:o[i + 1]].reshape(shapes[i]) for i in range(4)]


def make_step(cfg_dict, precision="fp32", rng="explicit", anchors=None, seed=0, splits=0):
    p = dadpkg.pkg()
    model = p.SSRLModel().cuda()
    view = p.ConfigView(cfg_dict, flavor=cfg_dict["flavor"])
    step = p.DADStep(model, view, precision=precision, rng=rng, anchors=anchors, seed=seed, splits=splits)
    return step


def load_state(step, st):
    """Seeded transition state (oracle/synth.make_state layout) -> device."""
    m = step.model
    with torch.no_grad():
        m.student_flat.copy_(torch.from_numpy(flat(st["student"])))
        m.teacher_flat.copy_(torch.from_numpy(flat(st["teacher"])))
        step.exp_avg.copy_(torch.from_numpy(flat(st["exp_avg"])))
        step.exp_avg_sq.copy_(torch.from_numpy(flat(st["exp_avg_sq"])))
        step.dacp[0:4].copy_(torch.from_numpy(np.asarray(st["tau"], np.float32)))
        step.dacp[4:8].copy_(torch.from_numpy(np.asarray(st["Q"], np.float32)))
    step.adam_step = int(st["nstep"])
    step.refresh_shadow()


def batches(inp):
    clean = {"net_input": {"feats": torch.from_numpy(inp["xc"]), "padding_mask": torch.from_numpy(inp["mc"])},
             "labels": torch.from_numpy(inp["yc"])}
    noisy = {"net_input": {"feats": torch.from_numpy(inp["xn"]), "padding_mask": torch.from_numpy(inp["mn"])},
             "labels": torch.from_numpy(inp["yn"])}
    draws = {k: inp[k] for k in ("nw", "ns", "u", "start", "keep1", "keep2")}
    return clean, noisy, draws


def run_step(step, inp, epoch, lr=None, with_draws=True):
    clean, noisy, draws = batches(inp)
    losses = step.step(clean, noisy, epoch, lr=lr, draws=draws if with_draws else None)
    torch.cuda.synchronize()
    Bc, Bn = inp["xc"].shape[0], inp["xn"].shape[0]
    out = {k: (v.detach().cpu().numpy() if torch.is_tensor(v) else v) for k, v in step.outputs(Bc, Bn).items()}
    out.update({k: float(v) for k, v in losses.items()})
    out["student"] = unflat(step.model.student_flat.detach().cpu().numpy())
    out["teacher"] = unflat(step.model.teacher_flat.detach().cpu().numpy())
    out["exp_avg"] = unflat(step.exp_avg.cpu().numpy())
    out["exp_avg_sq"] = unflat(step.exp_avg_sq.cpu().numpy())
    out["grads"] = unflat(out["grad"])
    out["dacp"] = step.dacp.cpu().numpy()
    return out


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    if a.size == 0:
        return 0.0
    return float(np.max(np.abs(a - b)) / max(1e-6, float(np.max(np.abs(b)))))


def close_grad(a, b, what, tol_norm=1e-4, tol_elem=1e-3):
    """Gradient / parameter check: Frobenius-relative <= tol_norm and max-relative <= tol_elem.

    The ReLU' pattern is a discrete decision: a pre-activation that rounds to ~0 can
    take the other sign on a different (equally valid) fp32 summation order, moving one
    row's contribution in one hidden unit's gradient row.  With ~1e6 decisions per
    branch per step that happens about once per B=64 step; it is visible elementwise but
    not in the norm, so gradients/parameters use a norm bound plus a looser elementwise one.
    """
    a = np.asarray(a, np.float64).reshape(-1)
    b = np.asarray(b, np.float64).reshape(-1)
    if a.size == 0:
        return
    rn = float(np.linalg.norm(a - b) / max(1e-12, float(np.linalg.norm(b))))
    if not rn < tol_norm:
        raise AssertionError("%s: norm-rel %.3e (tol %.1e)" % (what, rn, tol_norm))
    close(a, b, tol_elem, what + " [elementwise]")


def close(a, b, tol, what):
    """Max-relative check with a diagnostic message (index, values) on failure."""
    a = np.asarray(a, np.float64).reshape(-1)
    b = np.asarray(b, np.float64).reshape(-1)
    if a.size == 0:
        return
    err = np.abs(a - b)
    r = float(err.max() / max(1e-6, float(np.abs(b).max())))
    if not r < tol:
        i = int(err.argmax())
        raise AssertionError("%s: rel %.3e (tol %.1e) at %d: got %.9g want %.9g; max|want| %.6g; "
                             "n_bad(>tol) %d/%d" % (what, r, tol, i, a[i], b[i], np.abs(b).max(),
                                                    int((err > tol * np.abs(b).max()).sum()), a.size))
