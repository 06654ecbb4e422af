"""Eval path: validation metrics and anchor calibration on the device.

  validate            Trainer.validate                 I/train.py:522-564
  calibrate_anchors   Trainer._run_anchor_calibration  I/train.py:317-357
  predict_head        SSRLModel.predict + softmax + DACPManager.calculate_certainty_scores
                      (I/model.py:225-245, I/utils.py:401-430)

Every batch runs the HIP encoder forward (dad_encoder_forward, fp32 as the reference's eval) and
dad_predict_head (csrc/eval.hip: classifier, softmax, certainty score, argmax); predictions,
scores and labels stay on the device until one copy at the end of the loader, where the metrics
are computed with the same scikit-learn calls the reference makes.
"""
import numpy as np
import torch

from . import _lib
from .data import StoreFeats


def _feats_mask(batch, device):
    ni = batch["net_input"]
    x = ni["feats"]
    if isinstance(x, StoreFeats):
        x = x.materialize()
    x = x.to(device=device, dtype=torch.float32).contiguous()
    pm = ni.get("padding_mask")
    pad = (torch.zeros(x.shape[0], x.shape[1], dtype=torch.bool, device=device) if pm is None
           else pm.to(device=device, dtype=torch.bool).contiguous())
    return x, pad


def predict_head(model, x, padding_mask=None, use_teacher=False, use_entropy=True):
    """Eval-mode logits, softmax probs, certainty scores and argmax preds of one batch (device)."""
    enc = model.teacher_encoder if use_teacher else model.student_encoder
    cls = model.teacher_classifier if use_teacher else model.student_classifier
    with torch.no_grad():
        e = enc(x, padding_mask).contiguous()
        B = e.shape[0]
        out = {"logits": torch.empty(B, 4, device=e.device), "probs": torch.empty(B, 4, device=e.device),
               "score": torch.empty(B, device=e.device), "pred": torch.empty(B, dtype=torch.int64, device=e.device)}
        w2 = cls.fc_layer.weight.detach().contiguous()
        b2 = cls.fc_layer.bias.detach().contiguous()
        _lib.check(_lib.lib().dad_predict_head(
            _lib.ptr(e), B, _lib.ptr(w2), _lib.ptr(b2), int(bool(use_entropy)), _lib.ptr(out["logits"]),
            _lib.ptr(out["probs"]), _lib.ptr(out["score"]), _lib.ptr(out["pred"]),
            torch.cuda.current_stream(e.device).cuda_stream), "dad_predict_head")
    return out


def _collect(model, loader, use_teacher, want_labels, use_entropy=True):
    dev = model.student_flat.device
    preds, scores, labels = [], [], []
    for batch in loader:
        x, pad = _feats_mask(batch, dev)
        o = predict_head(model, x, pad, use_teacher=use_teacher, use_entropy=use_entropy)
        preds.append(o["pred"])
        scores.append(o["score"])
        if want_labels:
            labels.append(batch["labels"].to(device=dev, dtype=torch.int64))
    cat = lambda ts: torch.cat(ts).cpu().numpy() if ts else np.zeros(0)
    return cat(preds), cat(scores), (cat(labels) if want_labels else None)


def validate(model, data_loader, domain_name="unknown", num_classes=4, teacher_disagreement=False):
    """Trainer.validate (I/train.py:522-564): student predictions over the loader; with
    teacher_disagreement (the reference does it for noisy domains after warm-up) also the
    fraction of utterances where the teacher's argmax differs ('disagreement_rate')."""
    from sklearn.metrics import (accuracy_score, balanced_accuracy_score, confusion_matrix, f1_score,
                                 precision_recall_fscore_support)
    model.eval()
    preds, _, labels = _collect(model, data_loader, False, True)
    res = {}
    if teacher_disagreement:
        tp, _, _ = _collect(model, data_loader, True, False)
        if len(tp) == len(preds):
            res["disagreement_rate"] = float(np.mean(preds != tp))
    labs = range(num_classes)
    cm = confusion_matrix(labels, preds, labels=labs)
    prec, rec, f1, sup = precision_recall_fscore_support(labels, preds, average=None, zero_division=0, labels=labs)
    res.update({
        "accuracy": accuracy_score(labels, preds) * 100,
        "weighted_accuracy": balanced_accuracy_score(labels, preds) * 100,
        "f1_weighted": f1_score(labels, preds, average="weighted", zero_division=0) * 100,
        "f1_macro": f1_score(labels, preds, average="macro", zero_division=0) * 100,
        "precision_per_class": prec.tolist(), "recall_per_class": rec.tolist(),
        "f1_per_class": f1.tolist(), "support_per_class": sup.tolist(), "confusion_matrix": cm,
    })
    return res


def calibrate_anchors(model, clean_loader, noisy_loader, num_classes=4, anchor_std_k=1.5, use_entropy=True):
    """Trainer._run_anchor_calibration (I/train.py:317-357): per-class mean / std of the student's
    certainty scores on labeled clean and noisy data; anchors = clamp(mu_clean - k sigma_clean, 0)
    * mu_noisy / (mu_clean + 1e-8), float32 on the model's device (the `calibrated_anchors` input
    of DADStep).  Statistics in float64 over the float32 scores, as np.mean / np.std of .item()s."""
    model.eval()
    dev = model.student_flat.device
    stats = {}
    for name, loader in (("clean", clean_loader), ("noisy", noisy_loader)):
        _, s, y = _collect(model, loader, False, True, use_entropy=use_entropy)
        per = [s[y == c].astype(np.float64) for c in range(num_classes)]
        stats[name] = ([float(np.mean(v)) if len(v) else 0.0 for v in per],
                       [float(np.std(v)) if len(v) else 0.0 for v in per])
    mu_c = torch.tensor(stats["clean"][0], device=dev)
    mu_n = torch.tensor(stats["noisy"][0], device=dev)
    sd_c = torch.tensor(stats["clean"][1], device=dev)
    shift = mu_n / (mu_c + 1e-8)
    base = torch.clamp(mu_c - anchor_std_k * sd_c, min=0)
    model.train()
    return base * shift
