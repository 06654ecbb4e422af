"""Epoch-level state and checkpoint formats.

  train_epoch        Trainer.train_epoch loop + epoch end       I/train.py:474-520
  EarlyStopping      Trainer.check_early_stopping               I/train.py:566-579
  save_checkpoint    Trainer.save_checkpoint's dict             I/train.py:581-592
  load_checkpoint    (its inverse; weights_only unpickler)
  adam_state_dict    torch.optim.Adam(model.parameters()).state_dict() of the fused step's moments

The fused step keeps Adam's moments as flat device vectors in the [W1 | b1 | W2 | b2] order of
the student's parameters; a checkpoint stores them in torch.optim.Adam's own format over
SSRLModel.parameters() (8 tensors: the student's 4, then the teacher's 4, which never get a
gradient and so have no state), so a checkpoint written here loads into the reference's
optimizer and one written by the reference loads here.  The DACP state (ema_thresholds,
class_quality_scores, epoch statistics, anchors) rides along under 'dad_state'; the reference
does not save it, and a checkpoint without it leaves the step's DACP state untouched.
"""
import warnings

import numpy as np
import torch

from . import _lib

_SHAPES = [(256, 768), (256,), (4, 256), (4,)]
_SIZES = [256 * 768, 256, 4 * 256, 4]


def _split(flat):
    out, o = [], 0
    for n, s in zip(_SIZES, _SHAPES):
        out.append(flat[o:o + n].reshape(s))
        o += n
    return out


def adam_state_dict(exp_avg, exp_avg_sq, adam_step, lr, weight_decay, betas=(0.9, 0.999), eps=1e-8):
    """torch.optim.Adam(SSRLModel.parameters(), lr, weight_decay=...).state_dict() for flat
    moments of the student's parameters after `adam_step` steps (I/train.py:362)."""
    state = {}
    if adam_step > 0:
        for i, (m, v) in enumerate(zip(_split(exp_avg.detach().float().cpu()), _split(exp_avg_sq.detach().float().cpu()))):
            state[i] = {"step": torch.tensor(float(adam_step)), "exp_avg": m.clone(), "exp_avg_sq": v.clone()}
    group = {"lr": float(lr), "betas": tuple(betas), "eps": eps, "weight_decay": weight_decay, "amsgrad": False,
             "maximize": False, "foreach": None, "capturable": False, "differentiable": False, "fused": None,
             "decoupled_weight_decay": False, "params": list(range(8))}
    return {"state": state, "param_groups": [group]}


def load_adam_state_dict(sd, device):
    """(exp_avg, exp_avg_sq, adam_step, lr) flat on `device` from an Adam state dict over
    SSRLModel.parameters() (params 0-3 = the student's W1, b1, W2, b2)."""
    st = sd["state"]
    if any(k not in (0, 1, 2, 3) for k in st):
        raise ValueError("optimizer state for parameters other than the student's four")
    if not st:
        z = torch.zeros(_lib.DAD_NPARAM, device=device)
        return z, z.clone(), 0, float(sd["param_groups"][0]["lr"])
    steps = {float(st[i]["step"]) for i in st}
    if len(st) != 4 or len(steps) != 1:
        raise ValueError("expected one Adam step count over the student's four parameters")
    m = torch.cat([st[i]["exp_avg"].reshape(-1).float() for i in range(4)]).to(device)
    v = torch.cat([st[i]["exp_avg_sq"].reshape(-1).float() for i in range(4)]).to(device)
    return m, v, int(steps.pop()), float(sd["param_groups"][0]["lr"])


def _plain(results):
    """Validation dicts with their numpy confusion matrix as a list (weights_only-loadable)."""
    if results is None:
        return None
    return {k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in results.items()}


def save_checkpoint(path, epoch, model, step, clean_results=None, noisy_results=None, lr=None):
    """The reference's checkpoint dict (I/train.py:583): epoch, model_state_dict,
    optimizer_state_dict (torch Adam format), clean_results, noisy_results; plus dad_state."""
    view = step.view
    lr = view.lr_at(epoch) if lr is None else lr
    ckpt = {"epoch": epoch,
            "model_state_dict": {k: v.detach().cpu() for k, v in model.state_dict().items()},
            "optimizer_state_dict": adam_state_dict(step.exp_avg, step.exp_avg_sq, step.adam_step, lr,
                                                    view.WEIGHT_DECAY),
            "clean_results": _plain(clean_results), "noisy_results": _plain(noisy_results),
            "dad_state": {"dacp": step.dacp.detach().cpu(), "global_step": step.global_step}}
    torch.save(ckpt, path)
    return ckpt


def load_checkpoint(path, model, step=None):
    """Load a checkpoint written by save_checkpoint or by the reference's save_checkpoint into
    `model` (and the fused `step`: Adam moments, step count, DACP state).  Uses torch.load with
    weights_only=True; NumPy arrays in the results dicts (the reference's confusion matrices)
    are allowed through the weights-only unpickler's allowlist, nothing else."""
    allow = [np.ndarray, np.dtype, np._core.multiarray._reconstruct, np._core.multiarray.scalar] + \
        [type(np.dtype(t)) for t in (np.int64, np.float64, np.int32, np.float32, np.bool_)]
    with torch.serialization.safe_globals(allow):
        ckpt = torch.load(path, map_location="cpu", weights_only=True)
    with torch.no_grad():
        model.load_state_dict(ckpt["model_state_dict"])
    if step is not None:
        m, v, n, _ = load_adam_state_dict(ckpt["optimizer_state_dict"], step.device)
        step.exp_avg.copy_(m)
        step.exp_avg_sq.copy_(v)
        step.adam_step = n
        ds = ckpt.get("dad_state")
        if ds is not None:
            step.dacp.copy_(ds["dacp"].to(step.device))
            step.global_step = int(ds.get("global_step", step.global_step))
        step.refresh_shadow()
    return ckpt


class EarlyStopping:
    """Trainer.check_early_stopping (I/train.py:566-579): the caller says whether this epoch is
    the best so far (the reference compares the noisy domain's weighted accuracy); stop after
    `patience` epochs without improvement (EARLY_STOPPING / PATIENCE, I/config.py:146-147)."""

    def __init__(self, patience=50, enabled=True):
        self.patience = patience
        self.enabled = enabled
        self.patience_counter = 0

    def __call__(self, is_best):
        if not self.enabled:
            return False
        if is_best:
            self.patience_counter = 0
            return False
        self.patience_counter += 1
        return self.patience_counter >= self.patience


def train_epoch(step, clean_loader, noisy_loader, epoch, lr=None):
    """Trainer.train_epoch (I/train.py:474-520): min(len) batch pairs through the fused step at
    the epoch's cosine learning rate (CosineAnnealingLR(T_max=EPOCHS) stepped once per epoch),
    then the DACP epoch-end update after warm-up.  Returns the mean of each loss over the
    epoch (one device->host read, at the end).  Batches are drawn one ahead, so each step names
    the next one (16-bit modes prepare its rows inside the tail launch; the loaders hand out fresh
    device tensors per batch, and the results are the same either way)."""
    lr = step.view.lr_at(epoch) if lr is None else lr
    n = min(len(clean_loader), len(noisy_loader))
    ci, ni = iter(clean_loader), iter(noisy_loader)
    tot = None
    cur = (next(ci), next(ni)) if n else None
    for i in range(n):
        nxt = (next(ci), next(ni)) if i + 1 < n else None
        losses = step.step(cur[0], cur[1], epoch, lr=lr, next_batch=nxt)
        cur = nxt
        vec = torch.stack([losses[k].float().reshape(()) for k in sorted(losses)])
        tot = vec if tot is None else tot + vec
    if epoch >= step.view.WARMUP_EPOCHS:
        step.epoch_end()
    if tot is None:
        return {}
    # the range flag (dad.h DAD_T_RANGE, every batch shape's word) rides in the epoch's one
    # device->host read.  An encoder operand beyond +-65504 (FP16) or non-finite features make a
    # step's loss non-finite, which the reference's fp32 path cannot do: reported, and that step's
    # update skipped when its total loss is NaN.  A pooling hand-off timeout is a device fault, not
    # a data property: its steps' updates were skipped, and train_epoch raises.
    flag = step.range_flag(clear=True).float().reshape(1)
    vals = torch.cat([tot / n, flag]).cpu().tolist()
    out = dict(zip(sorted(losses), vals[:-1]))
    bits = int(vals[-1])
    out["range_flag"] = bits
    if bits & _lib.RANGE_POOL_TIMEOUT:
        raise RuntimeError("train_epoch(epoch=%d): the tail launch's pooling hand-off timed out in at least one "
                           "step (range flag %d); those steps' updates were skipped" % (epoch, bits))
    if bits & _lib.RANGE_NONFINITE:
        warnings.warn("train_epoch(epoch=%d): non-finite embeddings or logits in this epoch (fp16 operand "
                      "range exceeded or non-finite features); steps with a non-finite total loss were not applied"
                      % epoch, RuntimeWarning)
    return out
