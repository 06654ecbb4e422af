"""The helper-type drop-ins (DataAugmentation, DACPManager, ECDALoss; I/utils.py:317-652) on
the GPU, replayed against the reference's golden steps and the oracle.

  * DataAugmentation with the injected draws == the oracle's augmentation, bit for bit
    (3-D and 2-D inputs); with counter draws == the fused step's draws (dad_rng_draws).
  * DACPManager.calculate_mask on the reference's teacher probabilities (softmax of the
    golden teacher logits, on the CPU like the reference) reproduces the golden mask, scores,
    class weights and updated thresholds; the epoch update reproduces the golden Q.
  * ECDALoss on the golden embeddings reproduces the golden ecda_loss (1e-4) and the oracle's
    analytic gradients; the autograd path delivers them to the caller's tensors.
"""
import numpy as np
import pytest
import torch

import dadpkg
import gpu_harness as gh
import goldens
from oracle import dad_oracle, synth

pytestmark = pytest.mark.gpu
PKG = dadpkg.pkg()

DACP_VARIANTS = [n for n in goldens.variants() if not n.endswith(("fixed_thr", "fixed_ecda")) and
                 not n.startswith("casia_default")]
def _has_ecda(name):
    d = goldens.load(name)[0]
    return any(float(d["s%d_ecda_loss" % s]) != 0.0 for s in range(int(d["n_steps"])))


ECDA_VARIANTS = [n for n in goldens.variants() if _has_ecda(n)]


def _cuda(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    return t.to("cuda", dtype) if dtype is not None else t.cuda()


def _post_steps(d):
    return [(s, e) for s, e in goldens.schedule(d) if e >= 30 and ("s%d_e_teacher" % s) in d]


@pytest.mark.parametrize("name", ["iemocap_default", "emodb_b8", "iemocap_t300"])
def test_augmentation_explicit_draws_match_oracle(name):
    d, spec, cfg = goldens.load(name)
    aug = PKG.DataAugmentation(cfg=PKG.ConfigView(cfg, flavor=cfg["flavor"]))
    for s, _ in _post_steps(d)[:2]:
        inp = goldens.step_inputs(spec, s)
        x = _cuda(inp["xn"])
        w = aug.weak_augment(x, noise=inp["nw"]).cpu().numpy()
        st = aug.strong_augment(x, noise=inp["ns"], u=inp["u"], start=inp["start"]).cpu().numpy()
        np.testing.assert_array_equal(w, dad_oracle.weak_augment(inp["xn"], inp["nw"], cfg["WEAK_NOISE_STD"]))
        want = dad_oracle.strong_augment(inp["xn"], inp["ns"], inp["u"], inp["start"], cfg["STRONG_NOISE_STD"],
                                         cfg["DROPOUT_RATE"], cfg["TEMPORAL_MASK_RATIO"])
        np.testing.assert_array_equal(st, want)
        # 2-D [T, D] input: one start (I/utils.py:354-362)
        x2 = inp["xn"][0]
        st2 = aug.strong_augment(_cuda(x2), noise=inp["ns"][0], u=inp["u"], start=inp["start"][:1]).cpu().numpy()
        want2 = dad_oracle.strong_augment(x2[None], inp["ns"][:1], inp["u"], inp["start"][:1], cfg["STRONG_NOISE_STD"],
                                          cfg["DROPOUT_RATE"], cfg["TEMPORAL_MASK_RATIO"])[0]
        np.testing.assert_array_equal(st2, want2)
        # temporal masking alone
        tm = aug._apply_temporal_masking(x, start=inp["start"]).cpu().numpy()
        want3 = inp["xn"].copy()
        mlen = int(inp["xn"].shape[1] * cfg["TEMPORAL_MASK_RATIO"])
        for b in range(want3.shape[0]):
            want3[b, inp["start"][b]:inp["start"][b] + mlen] = 0
        np.testing.assert_array_equal(tm, want3)


def test_augmentation_counter_draws_are_the_step_s():
    B, T = 6, 50
    model = PKG.SSRLModel().cuda()
    step = PKG.DADStep(model, flavor="iemocap", precision="bf16", rng="counter", seed=99)
    aug = PKG.DataAugmentation(seed=99)
    aug.counter = 0
    x = torch.randn(B, T, 768, device="cuda")
    weak = aug.weak_augment(x)
    aug.counter = 0
    strong = aug.strong_augment(x)
    nw = step.counter_draws("weak", B, T, B, T, counter=0).view(B, T, 768)
    ns = step.counter_draws("strong", B, T, B, T, counter=0).view(B, T, 768)
    keep = step.counter_draws("feat_keep", B, T, B, T, counter=0)
    st = step.counter_draws("tstart", B, T, B, T, counter=0).long().cpu()
    assert torch.equal(weak, x + nw)
    want = (x + ns) * keep
    for b in range(B):
        want[b, st[b]:st[b] + 5] = 0
    assert torch.equal(strong, want)


def _probs(d, s):
    return torch.softmax(torch.from_numpy(d["s%d_z_teacher" % s]), dim=1)     # CPU float32, as the reference


@pytest.mark.parametrize("name", DACP_VARIANTS)
def test_dacp_manager_replays_goldens(name):
    d, spec, cfg = goldens.load(name)
    view = PKG.ConfigView(cfg, flavor=cfg["flavor"])
    mgr = PKG.DACPManager(4, cfg["EPOCHS"], "cuda", cfg=view)
    anchors = torch.from_numpy(np.asarray(spec.get("anchors", [0.0] * 4), np.float32))
    steps = [(s, e) for s, e in _post_steps(d) if ("s%d_mask" % s) in d]
    assert steps
    for s, epoch in steps:
        st = goldens.state(spec, s)
        mgr.ema_thresholds = st["tau"]
        mgr.class_quality_scores = st["Q"]
        q = _probs(d, s)
        mask, score, w = mgr.calculate_mask(q.cuda(), epoch, anchors)
        np.testing.assert_array_equal(mask.cpu().numpy(), d["s%d_mask" % s] > 0)
        gh.close(score.cpu().numpy(), d["s%d_score" % s], 1e-6, "%s score" % name)
        gh.close(w.cpu().numpy(), d["s%d_w" % s], 1e-6, "%s w" % name)
        gh.close(mgr.ema_thresholds.cpu().numpy(), d["s%d_tau_after" % s], 1e-6, "%s tau" % name)
        s2, p2 = PKG.DACPManager.calculate_certainty_scores(q.cuda(), cfg=view)
        so, po = dad_oracle.certainty_scores(q.numpy(), view.effective_switches()[2])
        np.testing.assert_array_equal(p2.cpu().numpy(), po)
        gh.close(s2.cpu().numpy(), so, 1e-6, "certainty")
    if "epoch_end_Q" in d:
        lists = mgr.batch_scores_per_class
        assert [len(v) for v in lists] == list(d["epoch_end_counts"])
        mgr.class_quality_scores = goldens.state(spec, int(d["epoch_end_after_step"]))["Q"]
        mgr.update_class_quality_scores_epoch(mgr.batch_scores_per_class)
        gh.close(mgr.class_quality_scores.cpu().numpy(), d["epoch_end_Q"], 1e-6, "%s epoch Q" % name)
        assert [len(v) for v in mgr.batch_scores_per_class] == [0, 0, 0, 0]


@pytest.mark.parametrize("name", ECDA_VARIANTS)
def test_ecda_loss_replays_goldens(name):
    d, spec, cfg = goldens.load(name)
    view = PKG.ConfigView(cfg, flavor=cfg["flavor"])
    use_dacp, use_ecda, use_entropy, class_aware = view.effective_switches()
    crit = PKG.ECDALoss(cfg=view)
    checked = 0
    for s, epoch in _post_steps(d):
        if float(d["s%d_ecda_loss" % s]) == 0.0:
            continue
        inp = goldens.step_inputs(spec, s)
        q = _probs(d, s)
        pred = q.argmax(1)
        if use_dacp:
            mask = torch.from_numpy(d["s%d_mask" % s] > 0)
            score = torch.from_numpy(d["s%d_score" % s])
            w = torch.from_numpy(d["s%d_w" % s])
        else:
            score = q.max(1).values
            mask = (score >= cfg["FIXED_CONFIDENCE_THRESHOLD"]).float()
            w = torch.ones_like(mask)
        ec = _cuda(d["s%d_e_clean" % s]).requires_grad_(True)
        es = _cuda(d["s%d_e_strong" % s]).requires_grad_(True)
        loss = crit(ec, es, _cuda(inp["yc"]), pred.cuda(), mask.cuda(), score.cuda(), w.cuda())
        want = float(d["s%d_ecda_loss" % s])
        assert abs(float(loss) - want) <= 1e-4 * max(1.0, abs(want)), (name, s, float(loss), want)
        loss.backward()
        tot, gec, ges = dad_oracle.ecda_loss(d["s%d_e_clean" % s], d["s%d_e_strong" % s], inp["yc"], pred.numpy(),
                                             mask.numpy(), score.numpy(), w.numpy(), cfg, class_aware, not use_dacp)
        gh.close_grad(ec.grad.cpu().numpy(), gec, "%s step %d d/d clean" % (name, s))
        gh.close_grad(es.grad.cpu().numpy(), ges, "%s step %d d/d noisy" % (name, s))
        checked += 1
    assert checked > 0
