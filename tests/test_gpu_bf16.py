"""BF16 throughput mode (the W-stationary encoder, csrc/encode_ws.hip) against FP32.

Two references:
  * the NumPy oracle with the reference's injected draws (rng='explicit'), on the edge
    geometries of test_gpu_parity (ragged lengths, slab-boundary crossings, Bc != Bn,
    Tc != Tn, warm-up and post-warm-up) -- checks the augmentation, the encoder, the
    pooling and the slab bookkeeping of the bf16 path;
  * the FP32 parity-mode kernels driven by the SAME counter RNG (rng='counter') -- the
    benchmark's configuration, including the in-kernel noise, feature mask and temporal
    mask, at the bench geometry B=64, T=300.
Tolerance: bf16 operands with fp32 accumulation -> embeddings/logits within 2e-2 of the
tensor max; gradient direction cosine > 0.99 whenever the discrete DACP mask agrees.
"""
import numpy as np
import pytest

import gpu_harness as gh
from oracle import dad_oracle, synth
from test_gpu_parity import EDGE, _problem

pytestmark = pytest.mark.gpu
BF16_TOL = 2e-2


def _grad_cos(g1, g2):
    a = np.concatenate([x.reshape(-1) for x in g1]).astype(np.float64)
    b = np.concatenate([x.reshape(-1) for x in g2]).astype(np.float64)
    return float(a @ b / max(1e-30, np.linalg.norm(a) * np.linalg.norm(b)))


@pytest.mark.parametrize("geom", EDGE, ids=lambda g: "B%dT%d_Bn%dTn%d" % (g["B"], g["T"], g["Bn"], g["Tn"]))
def test_bf16_step_edge_geometries_vs_oracle(geom):
    cfg = dad_oracle.make_cfg("iemocap")
    g = dict(geom)
    ragged = g.pop("ragged", True)
    inp = _problem(ragged=ragged, **g)
    st = synth.make_state(3, 1)
    step = gh.make_step(cfg, precision="bf16")
    orc = dad_oracle.DADOracle(*synth.init_weights(3)[:4], cfg)
    for epoch in (0, 60):
        gh.load_state(step, st)
        orc.load_state(st)
        o = gh.run_step(step, inp, epoch)
        r = orc.step(inp, epoch)
        gh.close(o["e_clean"], r["e_clean"], BF16_TOL, "%s e%d e_clean" % (geom, epoch))
        gh.close(o["z_clean"], r["z_clean"], BF16_TOL, "%s e%d z_clean" % (geom, epoch))
        if epoch >= 30:
            gh.close(o["e_teacher"], r["e_teacher"], BF16_TOL, "%s e_teacher" % (geom,))
            gh.close(o["e_strong"], r["e_strong"], BF16_TOL, "%s e_strong" % (geom,))
            gh.close(o["z_strong"], r["z_strong"], BF16_TOL, "%s z_strong" % (geom,))
        if epoch < 30 or np.array_equal(o["mask"], r["mask"]):
            assert _grad_cos(o["grads"], r["grads"]) > 0.99, (geom, epoch)


@pytest.mark.parametrize("B,T", [(16, 100), (64, 300)])
def test_bf16_counter_rng_matches_fp32_counter_rng(B, T):
    """Same seed -> same in-kernel noise, feature mask, temporal mask and dropout in both modes."""
    cfg = dad_oracle.make_cfg("iemocap")
    inp = _problem(B=B, T=T, seed=4, ragged=True)
    st = synth.make_state(4, 1)
    outs = []
    for prec in ("fp32", "bf16"):
        step = gh.make_step(cfg, precision=prec, rng="counter", seed=77)
        gh.load_state(step, st)
        outs.append(gh.run_step(step, inp, 60, with_draws=False))
    f, b = outs
    for k in ("e_clean", "e_teacher", "e_strong", "z_clean", "z_teacher", "z_strong"):
        gh.close(b[k], f[k], BF16_TOL, "counter %s B%d T%d" % (k, B, T))
    # the discrete DACP decisions agree at this geometry (a flip would move KL / ECDA by a
    # finite step, which no precision bound covers); then every loss term is within the bf16
    # loss bound of test_gpu_bf16_parity (the golden replays of the same mode)
    from test_gpu_bf16_parity import BF16_LOSS_TOL
    assert np.array_equal(b["mask"], f["mask"]), "bf16 and fp32 DACP masks differ (B%d T%d)" % (B, T)
    assert _grad_cos(b["grads"], f["grads"]) > 0.99
    for k in ("total_loss", "supervised_ce_loss", "consistency_loss", "ecda_loss"):
        err = abs(b[k] - f[k]) / max(1.0, abs(f[k]))
        print("counter B%d T%d %s: bf16 %.7g fp32 %.7g rel %.3g" % (B, T, k, b[k], f[k], err))
        assert err <= BF16_LOSS_TOL, (k, b[k], f[k], err)
    assert f["ecda_loss"] != 0.0 and f["consistency_loss"] != 0.0


def test_bf16_counter_steps_stay_finite():
    cfg = dad_oracle.make_cfg("iemocap")
    step = gh.make_step(cfg, precision="bf16", rng="counter", seed=3)
    gh.load_state(step, synth.make_state(6, 1))
    for k in range(4):
        inp = _problem(B=24, T=70, seed=10 + k, Bn=20, Tn=90)
        o = gh.run_step(step, inp, 40 + k, with_draws=False)
        assert all(np.isfinite(o[n]) for n in ("total_loss", "supervised_ce_loss", "consistency_loss", "ecda_loss"))
        assert all(np.all(np.isfinite(p)) for p in o["student"])


def test_bf16_factorised_weight_gradient_matches_direct(monkeypatch):
    """DAD_WGRAD=su (S_u = bits_u^T X_u on the side stream, then the dL/de-weighted sum) and
    the default direct GEMM compute the same dW1 from the same bf16 operands."""
    cfg = dad_oracle.make_cfg("iemocap")
    inp = _problem(B=20, T=90, seed=8, Bn=18, Tn=110, ragged=True)
    st = synth.make_state(8, 1)
    outs = []
    for mode in ("direct", "su"):
        monkeypatch.setenv("DAD_WGRAD", mode)
        step = gh.make_step(cfg, precision="bf16", rng="counter", seed=5)
        gh.load_state(step, st)
        outs.append(gh.run_step(step, inp, 60, with_draws=False))
    d, s = outs
    assert np.array_equal(d["mask"], s["mask"])
    for gd, gs in zip(d["grads"], s["grads"]):
        gh.close(gs, gd, BF16_TOL, "factorised vs direct grad")
    assert _grad_cos(d["grads"], s["grads"]) > 0.999


def test_bf16_shadow_follows_parameter_changes():
    """Parameters changed after the DADStep exists (load_state_dict, update_teacher_ema) must
    reach the bf16 W1 shadows of the next step: same result as a freshly constructed step."""
    import torch
    cfg = dad_oracle.make_cfg("iemocap")
    inp = _problem(B=16, T=60, seed=12, ragged=True)
    st = synth.make_state(12, 1)
    other = synth.make_state(13, 1)
    a = gh.make_step(cfg, precision="bf16", rng="counter", seed=9)
    gh.load_state(a, st)
    gh.run_step(a, inp, 60, with_draws=False)           # shadows now derived from the updated st params
    m = a.model
    sd = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in zip(
        ["student_encoder.pre_net.weight", "student_encoder.pre_net.bias", "student_classifier.fc_layer.weight",
         "student_classifier.fc_layer.bias", "teacher_encoder.pre_net.weight", "teacher_encoder.pre_net.bias",
         "teacher_classifier.fc_layer.weight", "teacher_classifier.fc_layer.bias"],
        list(other["student"]) + list(other["teacher"]))}
    m.load_state_dict(sd)                                # no refresh_shadow() call on purpose
    m.update_teacher_ema()
    a.global_step = 0
    with torch.no_grad():
        a.exp_avg.copy_(torch.from_numpy(gh.flat(other["exp_avg"])))
        a.exp_avg_sq.copy_(torch.from_numpy(gh.flat(other["exp_avg_sq"])))
        a.dacp[0:4].copy_(torch.from_numpy(np.asarray(other["tau"], np.float32)))
        a.dacp[4:8].copy_(torch.from_numpy(np.asarray(other["Q"], np.float32)))
        a.dacp[8:16].zero_()
    a.adam_step = int(other["nstep"])
    b = gh.make_step(cfg, precision="bf16", rng="counter", seed=9)
    with torch.no_grad():
        b.model.student_flat.copy_(m.student_flat)
        b.model.teacher_flat.copy_(m.teacher_flat)
        b.exp_avg.copy_(a.exp_avg)
        b.exp_avg_sq.copy_(a.exp_avg_sq)
        b.dacp.copy_(a.dacp)
    b.adam_step = a.adam_step
    b.refresh_shadow()
    oa = gh.run_step(a, inp, 60, with_draws=False)
    ob = gh.run_step(b, inp, 60, with_draws=False)
    for k in ("e_clean", "e_teacher", "e_strong", "z_strong"):
        np.testing.assert_array_equal(oa[k], ob[k], err_msg=k)
    for pa, pb in zip(oa["student"], ob["student"]):
        np.testing.assert_array_equal(pa, pb)
