"""16-bit throughput modes (FP16 and BF16 operands: the W-stationary encoder, csrc/encode_ws.hip,
and the direct weight gradient, csrc/wgrad.hip) against FP32.

Two references:
  * the NumPy oracle with the reference's injected draws (rng='explicit'), on the edge
    geometries of test_gpu_parity (ragged lengths, slab-boundary crossings, Bc != Bn,
    Tc != Tn, warm-up and post-warm-up) -- checks the augmentation, the encoder, the
    pooling and the slab bookkeeping of the 16-bit paths;
  * the FP32 parity-mode kernels driven by the SAME counter RNG (rng='counter') -- the
    benchmark's configuration, including the in-kernel noise, feature mask and temporal
    mask, at the bench geometry B=64, T=300.
Tolerance: 16-bit operands with fp32 accumulation -> of the tensor max, embeddings within 1e-3
(fp16) / 2e-2 (bf16); logits within 2e-2 (bf16) and, fp16, 7e-4 (1.5e-3 for the one-frame
geometry B1T1, whose embedding is a single row's ReLU with nothing averaging the operand
rounding).  Measured fp16 logits on these synthetic problems (round 5): 1.23e-3 (B1T1), 6.3e-4
(B5T33), 3.3e-4 .. 3.7e-4 (T = 40 .. 64); fp16 rounds each operand by up to 2^-11 relative.
north_star's 1e-4 holds on the reference's own inputs: every golden replay of
test_gpu_throughput_parity (15 fixtures).  Gradient direction cosine > 0.99 whenever the
discrete DACP mask agrees; losses within the golden-replay bounds of test_gpu_throughput_parity.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

import gpu_harness as gh
from oracle import dad_oracle, synth
from test_gpu_parity import EDGE, _problem

pytestmark = pytest.mark.gpu
BF16_TOL = 2e-2
ACT_TOL = {"bf16": BF16_TOL, "fp16": 1e-3}      # embeddings e_*
LOGIT_TOL = {"bf16": BF16_TOL, "fp16": 7e-4}    # logits z_*


def _tol(prec, key, T=None):
    if key.startswith("z_"):
        return 1.5e-3 if (prec == "fp16" and T == 1) else LOGIT_TOL[prec]
    return ACT_TOL[prec]
PRECS = ["fp16", "bf16"]


def _grad_cos(g1, g2):
    a = np.concatenate([x.reshape(-1) for x in g1]).astype(np.float64)
    b = np.concatenate([x.reshape(-1) for x in g2]).astype(np.float64)
    return float(a @ b / max(1e-30, np.linalg.norm(a) * np.linalg.norm(b)))


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("geom", EDGE, ids=lambda g: "B%dT%d_Bn%dTn%d" % (g["B"], g["T"], g["Bn"], g["Tn"]))
def test_16bit_step_edge_geometries_vs_oracle(geom, prec):
    cfg = dad_oracle.make_cfg("iemocap")
    g = dict(geom)
    ragged = g.pop("ragged", True)
    inp = _problem(ragged=ragged, **g)
    st = synth.make_state(3, 1)
    step = gh.make_step(cfg, precision=prec)
    orc = dad_oracle.DADOracle(*synth.init_weights(3)[:4], cfg)
    for epoch in (0, 60):
        gh.load_state(step, st)
        orc.load_state(st)
        o = gh.run_step(step, inp, epoch)
        r = orc.step(inp, epoch)
        keys = ["e_clean", "z_clean"] + (["e_teacher", "e_strong", "z_strong", "z_teacher"] if epoch >= 30 else [])
        print("%s %s e%d: %s" % (prec, geom, epoch, {k: float("%.3g" % gh.rel(o[k], r[k])) for k in keys}))
        for k in keys:
            gh.close(o[k], r[k], _tol(prec, k, min(g["T"], g["Tn"])), "%s %s e%d %s" % (prec, geom, epoch, k))
        if epoch < 30 or np.array_equal(o["mask"], r["mask"]):
            assert _grad_cos(o["grads"], r["grads"]) > 0.99, (geom, epoch)


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("B,T", [(16, 100), (64, 300)])
def test_16bit_counter_rng_matches_fp32_counter_rng(B, T, prec):
    """Same seed -> same in-kernel noise, feature mask, temporal mask and dropout in both modes."""
    from test_gpu_throughput_parity import TOL
    cfg = dad_oracle.make_cfg("iemocap")
    inp = _problem(B=B, T=T, seed=4, ragged=True)
    st = synth.make_state(4, 1)
    outs = []
    for p in ("fp32", prec):
        step = gh.make_step(cfg, precision=p, rng="counter", seed=77)
        gh.load_state(step, st)
        outs.append(gh.run_step(step, inp, 60, with_draws=False))
    f, b = outs
    for k in ("e_clean", "e_teacher", "e_strong", "z_clean", "z_teacher", "z_strong"):
        gh.close(b[k], f[k], _tol(prec, k), "counter %s %s B%d T%d" % (prec, k, B, T))
    # the discrete DACP decisions agree at this geometry (a flip would move KL / ECDA by a
    # finite step, which no precision bound covers); then every loss term is within the loss
    # bound of test_gpu_throughput_parity (the golden replays of the same mode)
    assert np.array_equal(b["mask"], f["mask"]), "%s and fp32 DACP masks differ (B%d T%d)" % (prec, B, T)
    assert _grad_cos(b["grads"], f["grads"]) > 0.99
    for k in ("total_loss", "supervised_ce_loss", "consistency_loss", "ecda_loss"):
        err = abs(b[k] - f[k]) / max(1.0, abs(f[k]))
        print("counter B%d T%d %s: %s %.7g fp32 %.7g rel %.3g" % (B, T, k, prec, b[k], f[k], err))
        assert err <= TOL[prec]["loss"], (prec, k, b[k], f[k], err)
    assert f["ecda_loss"] != 0.0 and f["consistency_loss"] != 0.0


@pytest.mark.parametrize("prec", PRECS)
def test_16bit_counter_steps_stay_finite(prec):
    cfg = dad_oracle.make_cfg("iemocap")
    step = gh.make_step(cfg, precision=prec, rng="counter", seed=3)
    gh.load_state(step, synth.make_state(6, 1))
    for k in range(4):
        inp = _problem(B=24, T=70, seed=10 + k, Bn=20, Tn=90)
        o = gh.run_step(step, inp, 40 + k, with_draws=False)
        assert all(np.isfinite(o[n]) for n in ("total_loss", "supervised_ce_loss", "consistency_loss", "ecda_loss"))
        assert all(np.all(np.isfinite(p)) for p in o["student"])


def test_fp16_range_flag():
    """FP16 operands overflow beyond +-65504: the step reports it in the sticky range flag
    (dad.h DAD_T_RANGE) instead of training on silently clipped rows; in-range steps leave it 0."""
    import torch
    cfg = dad_oracle.make_cfg("iemocap")
    inp = _problem(B=8, T=40, seed=21, ragged=True)
    step = gh.make_step(cfg, precision="fp16", rng="counter", seed=2)
    gh.load_state(step, synth.make_state(21, 1))
    gh.run_step(step, inp, 60, with_draws=False)
    assert int(step.range_flag()) == 0
    big = dict(inp)
    big["xc"] = inp["xc"].copy()
    big["xc"][1, 3, 17] = 1.0e5                            # one feature beyond the fp16 range
    gh.run_step(step, big, 60, with_draws=False)
    assert int(step.range_flag(clear=True)) != 0
    assert int(step.range_flag()) == 0                     # cleared
    # (that step's loss was not finite, so its update poisoned the parameters: start over)
    gh.load_state(step, synth.make_state(21, 1))
    gh.run_step(step, inp, 60, with_draws=False)
    assert int(step.range_flag()) == 0
    torch.cuda.synchronize()


def test_range_flag_covers_every_batch_shape():
    """each (Bc, Bn) shape has its own tail buffer; range_flag() ORs the words of all
    of them, so a flag raised by a full-size batch is seen (and cleared) after a ragged last batch
    of another shape ran."""
    cfg = dad_oracle.make_cfg("iemocap")
    step = gh.make_step(cfg, precision="fp16", rng="counter", seed=2)
    gh.load_state(step, synth.make_state(21, 1))
    full = _problem(B=8, T=40, seed=21, ragged=True)
    big = dict(full)
    big["xc"] = full["xc"].copy()
    big["xc"][1, 3, 17] = 1.0e5                            # beyond the fp16 range: this shape's word
    gh.run_step(step, big, 60, with_draws=False)
    last = _problem(B=5, T=40, seed=22, ragged=True, Bn=3)  # the epoch's ragged last batch: another word
    gh.load_state(step, synth.make_state(21, 1))
    gh.run_step(step, last, 60, with_draws=False)
    v = int(step.range_flag(clear=True))
    assert v & 1 and step.decode_range_flag(v) == ["nonfinite"]
    assert int(step.range_flag()) == 0                     # every shape's word cleared
    gh.run_step(step, full, 60, with_draws=False)
    assert int(step.range_flag()) == 0


def test_nonfinite_total_loss_skips_the_update():
    """A step whose total loss is not finite (an FP16 operand overflow here; the tail launch's pooling
    timeout writes a NaN total on purpose) leaves the parameters, moments, teacher and DACP state
    untouched (dad_optim), and the next finite step trains as before."""
    import torch
    cfg = dad_oracle.make_cfg("iemocap")
    inp = _problem(B=8, T=40, seed=31, ragged=True)
    step = gh.make_step(cfg, precision="fp16", rng="counter", seed=4)
    gh.load_state(step, synth.make_state(31, 1))
    before = [t.detach().clone() for t in (step.model.student_flat, step.model.teacher_flat, step.exp_avg,
                                            step.exp_avg_sq, step.dacp)]
    bad = dict(inp)
    bad["xc"] = inp["xc"].copy()
    bad["xc"][0, 0, 5] = 1.0e5                             # beyond the fp16 range in a clean frame
    o = gh.run_step(step, bad, 60, with_draws=False)
    assert not np.isfinite(o["total_loss"])
    after = (step.model.student_flat, step.model.teacher_flat, step.exp_avg, step.exp_avg_sq, step.dacp)
    for b, a in zip(before, after):
        assert torch.equal(b, a)
    assert int(step.range_flag(clear=True)) & 1
    o = gh.run_step(step, inp, 60, with_draws=False)
    assert np.isfinite(o["total_loss"]) and all(np.all(np.isfinite(p)) for p in o["student"])


def test_general_tail_kernel_switch_matches_wave_centric():
    """DAD_TAIL_W=0 (read once per process) selects the general tail + ECDA launch for every batch;
    in a subprocess it reproduces the wave-centric launch's losses, mask and gradient on a
    golden replay (the switch has no other coverage: the default takes the wave-centric kernel
    for batches of at most 64 per side)."""
    here = os.path.dirname(os.path.abspath(__file__))
    code = ("import sys, json; sys.path.insert(0, %r); sys.path.insert(0, %r)\n"
            "import numpy as np, goldens, gpu_harness as gh\n"
            "d, spec, cfg = goldens.load('casia_ecda_snr5')\n"
            "step = gh.make_step(cfg, precision='fp32', anchors=d['anchors'])\n"
            "out = {}\n"
            "for s, epoch in goldens.schedule(d):\n"
            "    gh.load_state(step, goldens.state(spec, s))\n"
            "    o = gh.run_step(step, goldens.step_inputs(spec, s), epoch, lr=float(d['s%%d_lr' %% s]))\n"
            "    out['s%%d' %% s] = [o['total_loss'], o['ecda_loss'], o['consistency_loss'],\n"
            "                      [float(x) for x in o['mask']], float(np.linalg.norm(o['grads'][0]))]\n"
            "print('RESULT' + json.dumps(out))\n") % (here, os.path.dirname(here))
    res = {}
    for mode in ("1", "0"):
        env = dict(os.environ, DAD_TAIL_W=mode)
        r = subprocess.run([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                           text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-3000:]
        line = [x for x in r.stdout.splitlines() if x.startswith("RESULT")][-1]
        import json
        res[mode] = json.loads(line[len("RESULT"):])
    for s in res["1"]:
        a, b = res["1"][s], res["0"][s]
        assert a[3] == b[3], (s, "mask")
        for i in (0, 1, 2, 4):
            assert abs(a[i] - b[i]) <= 1e-4 * max(1.0, abs(b[i])), (s, i, a[i], b[i])


@pytest.mark.parametrize("prec", PRECS)
def test_16bit_shadow_follows_parameter_changes(prec):
    """Parameters changed after the DADStep exists (load_state_dict, update_teacher_ema) must
    reach the 16-bit W1 shadows of the next step: same result as a freshly constructed step."""
    import torch
    cfg = dad_oracle.make_cfg("iemocap")
    inp = _problem(B=16, T=60, seed=12, ragged=True)
    st = synth.make_state(12, 1)
    other = synth.make_state(13, 1)
    a = gh.make_step(cfg, precision=prec, rng="counter", seed=9)
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
    b = gh.make_step(cfg, precision=prec, rng="counter", seed=9)
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
