"""Loss parity of the BENCHMARKED modes: 16-bit MFMA operands (the W-stationary encoder and the
direct weight gradient) replayed against the reference's own goldens.

The bench line times the fp16 step (fp16 operands, fp32 accumulation; it also reports a bf16
leg).  Here each 16-bit step runs with the reference's injected draws (rng='explicit', so the
augmentation noise, feature mask, temporal mask and dropout masks are the reference's) from the
goldens' seeded states, and is compared with what the reference itself computed
(tests/golden/gen_golden.py) at
  * the bench geometry B=64, T=300 (iemocap_b64_t300: warm-up + two full-weight steps), and
  * BASELINE configs[3], CASIA with DACP + ECDA on at SNR 0 / 5 / 10 dB (casia_ecda_snr*),
on every term of the loss graph (I/train.py:462-466): total, CE, consistency KL, ECDA; the
student/teacher logits and embeddings; the DACP mask (bit-exact); the clipped gradients and
post-step parameters.

Tolerances:
  FP16 (the timed mode): north_star's bound, 1e-4, on every loss term and on the student and
    teacher logits; fp16 keeps 11 significand bits (operands rounded by up to 2^-12 relative).
    Measured (round 4, the 4 bench fixtures, all steps): losses <= 2.5e-5, logits <= 8.1e-5,
    embeddings <= 2.7e-4, clipped-gradient Frobenius <= 9.2e-3 (cosine 1.0; the gradient error is
    set by ReLU' decisions of pre-activations within rounding of 0, which flip whole rows),
    post-step parameters <= 1.2e-6; the DACP mask identical on every step.  The non-north-star
    bounds are about 3x those.  Round 5 replays every step fixture in fp16: the post-step
    parameters of EMODB (its learning rate and few rows per step) reach 1.01e-5, so their bound
    is 3e-5.
  BF16: 8 significand bits (2^-9).  Bounds about 3x the largest error measured on MI355X
    (round 3, all 4 fixtures, all steps: losses 1.5e-4, logits 5.4e-4, embeddings 2.3e-3,
    clipped-gradient Frobenius 2.2e-2 (cosine >= 0.99988), post-step parameters 2.1e-6).
  losses        |x - ref| <= LOSS_TOL * max(1, |ref|)
  logits        max-abs error <= LOGIT_TOL * max|ref|
  embeddings    max-abs error <= EMB_TOL * max|ref|
  gradients     Frobenius-relative <= GRAD_TOL; cosine >= GRAD_COS
  parameters    Frobenius-relative <= PARAM_TOL (one Adam step from the same state)
The tests print the measured errors; with DAD_PARITY_JSON set they are also written there.
"""
import json
import os

import numpy as np
import pytest

import goldens
import gpu_harness as gh

pytestmark = pytest.mark.gpu

GOLDENS = ["iemocap_b64_t300", "casia_ecda_snr0", "casia_ecda_snr5", "casia_ecda_snr10"]
TOL = {
    "fp16": {"loss": 1e-4, "logit": 1e-4, "emb": 1e-3, "grad": 3e-2, "cos": 0.9999, "param": 3e-5},
    "bf16": {"loss": 5e-4, "logit": 1.5e-3, "emb": 7e-3, "grad": 6e-2, "cos": 0.9995, "param": 1e-5},
}
BF16_LOSS_TOL = TOL["bf16"]["loss"]
_LOSSES = ("total_loss", "supervised_ce_loss", "consistency_loss", "ecda_loss")
_MEASURED = {}


def _normrel(a, b):
    a = np.asarray(a, np.float64).reshape(-1)
    b = np.asarray(b, np.float64).reshape(-1)
    return float(np.linalg.norm(a - b) / max(1e-30, float(np.linalg.norm(b))))


def _cos(a, b):
    a = np.asarray(a, np.float64).reshape(-1)
    b = np.asarray(b, np.float64).reshape(-1)
    return float(a @ b / max(1e-30, float(np.linalg.norm(a) * np.linalg.norm(b))))


def _record(prec, name, s, key, v):
    _MEASURED.setdefault(prec, {}).setdefault(name, {}).setdefault("s%d" % s, {})[key] = v


@pytest.fixture(scope="module", autouse=True)
def _dump_measured():
    yield
    path = os.environ.get("DAD_PARITY_JSON")
    if path and _MEASURED:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump(_MEASURED, f, indent=1, sort_keys=True)


# fp16 (the timed mode) on EVERY step fixture: besides the bench geometry and configs[3], the
# reference's other branches -- global MMD (I/utils.py:633-650), no-entropy certainty
# (I/utils.py:414), the fixed threshold (I/train.py:417-420), EMODB's unconditional DACP
# (E/train_emodb.py:419), mask-empty steps, Bc != Bn and T = 300 shapes -- at north_star's 1e-4.
# bf16 (a mode, not the headline) on the four bench fixtures.
CASES = [(n, "fp16") for n in goldens.variants()] + [(n, "bf16") for n in GOLDENS]


@pytest.mark.parametrize("name,prec", CASES, ids=["%s-%s" % c for c in CASES])
def test_16bit_step_matches_reference_goldens(name, prec):
    tol = TOL[prec]
    d, spec, cfg = goldens.load(name)
    step = gh.make_step(cfg, precision=prec, anchors=d["anchors"])
    idx = d["w1_index"]
    worst = {}
    for s, epoch in goldens.schedule(d):
        p = "s%d_" % s
        gh.load_state(step, goldens.state(spec, s))
        inp = goldens.step_inputs(spec, s)
        o = gh.run_step(step, inp, epoch, lr=float(d[p + "lr"]))
        errs = {}
        for k in _LOSSES:
            ref = float(d[p + k])
            errs[k] = abs(o[k] - ref) / max(1.0, abs(ref))
        acts = ["z_clean", "e_clean"] + (["z_strong", "z_teacher", "e_strong", "e_teacher"] if p + "z_strong" in d else [])
        for k in acts:
            errs[k] = gh.rel(o[k], d[p + k])
        mask_ok = True
        if p + "mask" in d:
            mask_ok = bool(np.array_equal(o["mask"], d[p + "mask"]))
            errs["mask_flips"] = int(np.sum(o["mask"] != d[p + "mask"]))
        coef = np.float32(o["clip_coef"])
        g = [x * coef for x in o["grads"]]
        gref = [d[p + "gW1c_s"], d[p + "gb1c"], d[p + "gW2c"], d[p + "gb2c"]]
        gget = [g[0].reshape(-1)[idx], g[1], g[2], g[3]]
        errs["grad_normrel"] = max(_normrel(a, b) for a, b in zip(gget, gref))
        errs["grad_cos"] = _cos(np.concatenate([x.reshape(-1) for x in gget]),
                                np.concatenate([np.asarray(x).reshape(-1) for x in gref]))
        prm = o["student"]
        errs["param_normrel"] = max(_normrel(prm[0].reshape(-1)[idx], d[p + "sW1_s"]), _normrel(prm[1], d[p + "sb1"]),
                                    _normrel(prm[2], d[p + "sW2"]), _normrel(prm[3], d[p + "sb2"]))
        for k, v in errs.items():
            _record(prec, name, s, k, v)
            if k == "grad_cos":
                worst[k] = min(worst.get(k, 1.0), v)
            else:
                worst[k] = max(worst.get(k, 0.0), v)
        print("%s %s step %d (epoch %d): %s" % (prec, name, s, epoch,
                                               json.dumps({k: float("%.3g" % v) for k, v in errs.items()})))
        assert mask_ok, (prec, name, s, "DACP mask differs from the reference", errs.get("mask_flips"))
        for k in _LOSSES:
            assert errs[k] <= tol["loss"], (prec, name, s, k, errs[k])
        for k in acts:
            assert errs[k] <= (tol["logit"] if k.startswith("z_") else tol["emb"]), (prec, name, s, k, errs[k])
        assert errs["grad_normrel"] <= tol["grad"], (prec, name, s, errs["grad_normrel"])
        assert errs["grad_cos"] >= tol["cos"], (prec, name, s, errs["grad_cos"])
        assert errs["param_normrel"] <= tol["param"], (prec, name, s, errs["param_normrel"])
        rf = int(step.range_flag())
        assert rf == 0, (prec, name, s, "range flag set on in-range features", rf)
    print("%s %s worst: %s" % (prec, name, json.dumps({k: float("%.3g" % v) for k, v in worst.items()})))
