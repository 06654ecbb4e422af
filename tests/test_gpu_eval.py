"""Eval path on the MI355X (evaluate.py + csrc/eval.hip) against the reference trainer's own
validate() and _run_anchor_calibration() (golden tests/golden/eval_iemocap.npz, made by
tests/golden/gen_data_golden.py on seeded synthetic files and weights), and the prediction head
against a torch fp32 restatement of the same op."""
import numpy as np
import pytest
import torch

import dadpkg
import gpu_harness as gh
from oracle import data_oracle as do
from test_data_cpu import _golden

pytestmark = pytest.mark.gpu
PKG = dadpkg.pkg()
D = PKG.data
E = PKG.evaluate


def _model(seed):
    stu, tea = do.eval_weights(seed)
    model = PKG.SSRLModel().cuda()
    with torch.no_grad():
        model.student_flat.copy_(torch.from_numpy(gh.flat(stu)))
        model.teacher_flat.copy_(torch.from_numpy(gh.flat(tea)))
    return model


def test_validate_and_calibration_match_reference(tmp_path):
    g = _golden("eval_iemocap")
    seed, bs, fold = int(g["seed"]), int(g["batch_size"]), int(g["fold"])
    do.write_synthetic_split(str(tmp_path), seed, n_utt=160, max_len=40, flavor="iemocap")
    model = _model(seed)
    _, cval, ctest, _, _ = D.get_cv_dataloaders(str(tmp_path), bs, fold_id=fold)
    nval = D.get_cv_dataloaders_noisy(str(tmp_path), bs, fold_id=fold)[2]
    for name, ld, noisy in (("clean_val", cval, False), ("clean_test", ctest, False), ("noisy_val", nval, True)):
        r = E.validate(model, ld, teacher_disagreement=noisy)
        for k in ("accuracy", "weighted_accuracy", "f1_weighted", "f1_macro"):
            assert r[k] == pytest.approx(float(g["%s_%s" % (name, k)]), abs=1e-9), (name, k)
        for k in ("precision_per_class", "recall_per_class", "f1_per_class", "support_per_class"):
            np.testing.assert_allclose(r[k], g["%s_%s" % (name, k)], atol=1e-12, err_msg="%s %s" % (name, k))
        np.testing.assert_array_equal(r["confusion_matrix"], g[name + "_confusion_matrix"])
        if noisy:
            assert r["disagreement_rate"] == pytest.approx(float(g["noisy_val_disagreement_rate"]), abs=1e-12)
    # calibration reads the clean TRAIN loader and the noisy VAL loader at twice the batch size
    ctrain = D.get_cv_dataloaders(str(tmp_path), 2 * bs, fold_id=fold)[0]
    ncal = D.get_cv_dataloaders_noisy(str(tmp_path), 2 * bs, fold_id=fold)[2]
    anchors = E.calibrate_anchors(model, ctrain, ncal, anchor_std_k=float(g["anchor_std_k"]))
    np.testing.assert_allclose(anchors.cpu().numpy(), g["calibrated_anchors"], rtol=1e-4, atol=1e-8)


@pytest.mark.parametrize("use_entropy", [True, False])
def test_predict_head_matches_torch_fp32(use_entropy):
    model = _model(11)
    rs = np.random.RandomState(12)
    B, T = 37, 23
    x = torch.from_numpy(rs.standard_normal((B, T, 768)).astype(np.float32)).cuda()
    pad = torch.from_numpy(rs.rand(B, T) < 0.2).cuda()
    pad[:, 0] = False
    for use_teacher in (False, True):
        o = E.predict_head(model, x, pad, use_teacher=use_teacher, use_entropy=use_entropy)
        enc = model.teacher_encoder if use_teacher else model.student_encoder
        cls = model.teacher_classifier if use_teacher else model.student_classifier
        with torch.no_grad():
            e = enc(x, pad)
            z = e @ cls.fc_layer.weight.T + cls.fc_layer.bias
            p = torch.softmax(z, dim=1)
            mp, pred = torch.max(p, dim=1)
            ent = -(p * torch.log2(p + 1e-8)).sum(1)
            sc = mp * (1 - ent / np.log2(4)) if use_entropy else mp
        torch.testing.assert_close(o["logits"], z, rtol=1e-5, atol=1e-4)
        torch.testing.assert_close(o["probs"], p, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(o["score"], sc, rtol=1e-5, atol=1e-6)
        assert torch.equal(o["pred"], pred)
        assert torch.equal(o["pred"], torch.argmax(o["logits"], 1))
