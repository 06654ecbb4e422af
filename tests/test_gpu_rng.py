"""Distribution of the throughput mode's counter-RNG draws (rng='counter').

The reference draws its augmentation and dropout from torch's generators (I/utils.py:330,338,
343,370; nn.Dropout, I/model.py:54-64).  The MI355X step draws them in-kernel from a keyed
hash (csrc/dad_common.h), so it matches the reference in distribution, not bit for bit.  These
tests read the draws through the C ABI's dad_rng_draws, which calls the same device functions
the step kernels call, and check them against the reference's distributions:

  * weak / strong noise over >= 1.4e7 samples: mean, std, KS statistic against N(0, 1),
    tail mass beyond 3 sigma, lag correlations, weak-vs-strong correlation, and across steps;
  * feature keep rate 0.9 (one [768] mask per step, shared by the batch);
  * temporal-mask starts uniform over [0, Tmax - floor(0.1 Tmax)] (chi-square);
  * classifier dropout: factors exactly 0 or float32(1/0.9), keep rate 0.9, the two passes
    independent.
Significance: 5-sigma bounds / p > 1e-4, so a correct generator fails with negligible odds.
"""
import math

import numpy as np
import pytest
import torch

import dadpkg

pytestmark = pytest.mark.gpu
PKG = dadpkg.pkg()
B, T = 64, 300


@pytest.fixture(scope="module")
def step():
    model = PKG.SSRLModel().cuda()
    return PKG.DADStep(model, flavor="iemocap", precision="bf16", rng="counter", seed=20260101)


def _z(step, which, counter=0):
    v = step.counter_draws(which, B, T, B, T, counter=counter).double()
    std = 0.01 if which == "weak" else 0.05
    return (v / std).cpu().numpy()


def _ks_normal(z):
    from scipy.special import ndtr
    zs = np.sort(z)
    n = zs.size
    cdf = ndtr(zs)
    i = np.arange(1, n + 1)
    return float(max(np.max(i / n - cdf), np.max(cdf - (i - 1) / n)))


@pytest.mark.parametrize("which", ["weak", "strong"])
def test_noise_is_standard_normal(step, which):
    z = np.concatenate([_z(step, which, c) for c in (0, 1)])     # 2 x 14.7e6 samples
    n = z.size
    assert n >= 1.4e7
    tol = 5.0 / math.sqrt(n)
    assert abs(z.mean()) < tol, z.mean()
    assert abs(z.std() - 1.0) < 5.0 * math.sqrt(0.5 / n) + 1e-4, z.std()
    ks = _ks_normal(z)
    assert ks < 1.95 / math.sqrt(n) * 1.5, ks            # alpha ~ 1e-3 critical value, with margin
    # tail mass beyond 3 sigma (Box-Muller truncates at 4.71 sigma: mass 2.5e-6 lost)
    p3 = 2 * 0.0013498980316301
    f3 = float(np.mean(np.abs(z) > 3.0))
    assert abs(f3 - p3) < 5 * math.sqrt(p3 * (1 - p3) / n), (f3, p3)
    assert np.max(np.abs(z)) < 4.72
    # kurtosis of a normal: 3
    k = float(np.mean(z ** 4))
    assert abs(k - 3.0) < 5 * math.sqrt(96.0 / n), k
    # no correlation between neighbours (the two normals of one hash), across a row, across steps
    zz = z[: n // 2]
    for lag in (1, 2, 768, 768 * 300):
        c = float(np.corrcoef(zz[:-lag], zz[lag:])[0, 1])
        assert abs(c) < 5.0 / math.sqrt(zz.size - lag), (lag, c)
    c = float(np.corrcoef(z[: n // 2], z[n // 2:])[0, 1])
    assert abs(c) < 5.0 / math.sqrt(n // 2), ("step 0 vs step 1", c)


def test_weak_and_strong_streams_independent(step):
    w, s = _z(step, "weak"), _z(step, "strong")
    c = float(np.corrcoef(w, s)[0, 1])
    assert abs(c) < 5.0 / math.sqrt(w.size), c


def test_noise_scaled_by_config_std(step):
    w = step.counter_draws("weak", B, 40, B, 40).double().cpu().numpy()
    s = step.counter_draws("strong", B, 40, B, 40).double().cpu().numpy()
    n = w.size
    assert abs(w.std() / 0.01 - 1) < 5 * math.sqrt(0.5 / n) + 1e-4
    assert abs(s.std() / 0.05 - 1) < 5 * math.sqrt(0.5 / n) + 1e-4


def test_feature_keep_rate(step):
    steps = 2000
    k = torch.stack([step.counter_draws("feat_keep", B, T, B, T, counter=c) for c in range(steps)]).cpu().numpy()
    assert set(np.unique(k)) <= {0.0, 1.0}
    n = k.size
    rate = float(k.mean())
    assert abs(rate - 0.9) < 3 * math.sqrt(0.09 / n) * 1.67, rate      # 5 sigma
    # every channel is dropped at the same rate (no channel-dependent bias)
    per_ch = k.mean(0)
    assert np.all(np.abs(per_ch - 0.9) < 5 * math.sqrt(0.09 / steps)), per_ch.min()
    # masks of consecutive steps independent
    c = float(np.corrcoef(k[:-1].reshape(-1), k[1:].reshape(-1))[0, 1])
    assert abs(c) < 5.0 / math.sqrt(k[:-1].size), c


def test_temporal_start_uniform(step):
    from scipy.stats import chi2
    mlen = int(T * 0.1)
    hi = T - mlen + 1                      # randint(0, max(1, Tmax - mask_len + 1))
    steps = 4000
    st = torch.cat([step.counter_draws("tstart", B, T, B, T, counter=c) for c in range(steps)]).cpu().numpy()
    assert st.min() >= 0 and st.max() <= hi - 1 and np.all(st == np.round(st))
    h = np.bincount(st.astype(np.int64), minlength=hi)
    assert h.size == hi
    exp = st.size / hi
    x2 = float(((h - exp) ** 2 / exp).sum())
    assert chi2.sf(x2, hi - 1) > 1e-4, x2
    assert abs(st.mean() - (hi - 1) / 2) < 5 * math.sqrt((hi * hi - 1) / 12 / st.size)
    # short sequences: mask_len 0 -> start_hi = Tn + 1 ... and Tn = 5 -> hi = 6 (int(0.5) = 0)
    s5 = torch.cat([step.counter_draws("tstart", B, 5, B, 5, counter=c) for c in range(500)]).cpu().numpy()
    assert set(np.unique(s5)) == set(range(6))


@pytest.mark.parametrize("which", ["keep1", "keep2"])
def test_classifier_dropout_keep_rate(step, which):
    steps = 200
    k = torch.cat([step.counter_draws(which, B, T, B, T, counter=c) for c in range(steps)]).cpu().numpy()
    scale = np.float32(1.0) / np.float32(0.9)
    assert set(np.unique(k)) == {0.0, float(scale)}
    keep = k > 0
    n = keep.size
    assert abs(keep.mean() - 0.9) < 5 * math.sqrt(0.09 / n), keep.mean()


def test_dropout_passes_independent(step):
    k1 = step.counter_draws("keep1", B, T, B, T).cpu().numpy() > 0
    k2 = step.counter_draws("keep2", B, T, B, T).cpu().numpy() > 0
    c = float(np.corrcoef(k1, k2)[0, 1])
    assert abs(c) < 5.0 / math.sqrt(k1.size), c


def test_draws_are_the_step_s_draws():
    """The probe and the step kernels draw the same values: a bf16 counter-RNG step and a bf16
    explicit-draw step fed the probe's draws (noise / std, keep flags as u, starts, dropout
    masks) give the same embeddings and logits.  The clean pass (dropout #1 only) is bit-exact;
    the noisy passes differ only by the rounding of (noise / std) * std."""
    import gpu_harness as gh
    from oracle import dad_oracle, synth
    cfg = dad_oracle.make_cfg("iemocap")
    Bc, Tc, Bn, Tn = 12, 70, 10, 90
    inp = synth.make_step_inputs(5, 0, Bc, Tc)
    inpn = synth.make_step_inputs(6, 0, Bn, Tn)
    inp.update(xn=inpn["xn"], mn=inpn["mn"], yn=inpn["yn"])
    st = synth.make_state(5, 1)
    a = gh.make_step(cfg, precision="bf16", rng="counter", seed=4242)
    gh.load_state(a, st)
    d = {k: a.counter_draws(k, Bc, Tc, Bn, Tn).cpu().numpy() for k in
         ("weak", "strong", "feat_keep", "tstart", "keep1", "keep2")}
    oa = gh.run_step(a, inp, 60, with_draws=False)
    b = gh.make_step(cfg, precision="bf16", rng="explicit")
    gh.load_state(b, st)
    draws = {"nw": (d["weak"] / np.float32(0.01)).reshape(Bn, Tn, 768),
             "ns": (d["strong"] / np.float32(0.05)).reshape(Bn, Tn, 768),
             "u": d["feat_keep"].astype(np.float32), "start": d["tstart"].astype(np.int64),
             "keep1": (d["keep1"] > 0).reshape(Bc, 256), "keep2": (d["keep2"] > 0).reshape(Bn, 256)}
    clean, noisy, _ = gh.batches(inp)
    b.step(clean, noisy, 60, draws=draws)
    torch.cuda.synchronize()
    ob = {k: (v.detach().cpu().numpy() if torch.is_tensor(v) else v) for k, v in b.outputs(Bc, Bn).items()}
    np.testing.assert_array_equal(oa["e_clean"], ob["e_clean"])
    np.testing.assert_array_equal(oa["z_clean"], ob["z_clean"])
    for k in ("e_teacher", "e_strong", "z_teacher", "z_strong"):
        gh.close(oa[k], ob[k], 2e-3, "counter vs explicit-with-probe-draws " + k)
    np.testing.assert_array_equal(oa["mask"], ob["mask"])
