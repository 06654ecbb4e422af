"""Next-batch row preparation inside the tail launch (DADStep.step(next_batch=...), C ABI
dad_step_backward_ahead + dad_config.prepped).

The 16-bit steps' augmentation and conversion (dad_prep.h) are weight-independent, so a step can
prepare the NEXT batch's rows on the CUs its tail launch leaves idle.  A chain of steps over
rotating device-resident batches that names each next batch must equal the same chain without it
bit for bit (same RNG streams, same bytes, same GEMMs); the later steps must really have skipped
their own preparation; a step whose batch is not the one named falls back to preparing itself."""
import numpy as np
import pytest
import torch

import gpu_harness as gh
from oracle import dad_oracle, synth
from test_gpu_graph import _device_batches, _state
from test_gpu_parity import _problem

pytestmark = pytest.mark.gpu
K = 7


def _chain(cfg, precision, batches, st, ahead, wrong_at=None, split=False):
    step = gh.make_step(cfg, precision=precision, rng="counter", seed=5)
    step.prep_under_exchange = split    # (the DP step's default: noisy rows on a side stream)
    gh.load_state(step, st)
    losses, prepped = [], []
    for k in range(K):
        c, n = batches[k % len(batches)]
        nxt = None
        if ahead:
            nxt = batches[(k + 1) % len(batches)] if k != wrong_at else batches[(k + 2) % len(batches)]
        out = step.step(c, n, 60, next_batch=nxt)
        losses.append({key: float(v) for key, v in out.items()})
        prepped.append(step.last_prepped)
    torch.cuda.synchronize()
    return _state(step), losses, prepped


@pytest.mark.parametrize("precision,B,T", [("fp16", 16, 40), ("bf16", 16, 40), ("fp16", 64, 300)])
def test_prefetch_chain_equals_plain_chain(precision, B, T):
    """(B=64, T=300: the bench geometry, 251 preparation workgroups in the tail launch.)"""
    cfg = dad_oracle.make_cfg("iemocap")
    Bn, Tn = (12, 50) if B == 16 else (B, T)
    batches = [_device_batches(_problem(B=B, T=T, seed=31 + i, Bn=Bn, Tn=Tn))[:2] for i in range(3)]
    st = synth.make_state(31, 1)
    want, want_losses, plain_prepped = _chain(cfg, precision, batches, st, ahead=False)
    assert not any(plain_prepped)
    got, got_losses, prepped = _chain(cfg, precision, batches, st, ahead=True, wrong_at=3)
    # step 0 prepares itself; steps 1..K-1 use the previous tail launch's rows, except step 4,
    # whose batch is not the one step 3 named (it prepares itself)
    assert prepped == [False, True, True, True, False, True, True], prepped
    for name, a, b in zip(("student", "teacher", "exp_avg", "exp_avg_sq", "dacp", "grad"), got, want):
        assert torch.equal(a, b), "%s differs (max %.3g)" % (name, float((a - b).abs().max()))
    assert got_losses == want_losses


def test_prefetch_refused_for_other_geometry():
    """A next batch of another shape is not prepared ahead (its set would not sit where the next
    step looks); the step runs as without it."""
    cfg = dad_oracle.make_cfg("iemocap")
    a = _device_batches(_problem(B=16, T=40, seed=41, Bn=12, Tn=50))[:2]
    b = _device_batches(_problem(B=16, T=44, seed=42, Bn=12, Tn=50))[:2]
    st = synth.make_state(41, 1)
    step = gh.make_step(cfg, precision="fp16", rng="counter", seed=5)
    gh.load_state(step, st)
    step.step(a[0], a[1], 60, next_batch=b)
    assert step._prepped_key is None
    step.step(b[0], b[1], 60)
    torch.cuda.synchronize()
    assert not step.last_prepped


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_prefetch_store_batches(precision):
    """Store-mode batches (rows gathered from a ragged FeatureStore, no padded copy) prepared ahead:
    the next batch's clean rows are converted inside the weight-gradient launch through the
    utterance table (dad_wgrad_direct*_cps), its noisy rows in the tail launch.  The chain equals
    the plain store chain and the padded (collated) chain bit for bit."""
    import dadpkg
    PKG = dadpkg.pkg()
    D = PKG.data
    cfg = dad_oracle.make_cfg("iemocap")
    rs = np.random.RandomState(52)
    n_utt = 96
    sizes = rs.randint(6, 41, size=n_utt)
    sizes[:4] = 40                                   # every batch below holds one 40-frame utterance
    feats = (rs.standard_normal((int(sizes.sum()), 768)) * 0.5).astype("float32")
    offsets = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    store = D.FeatureStore(feats, sizes, offsets, rs.randint(0, 4, size=n_utt))
    picks = []
    for i in range(3):
        ic = np.concatenate([[i], 4 + rs.choice(n_utt - 4, 15, replace=False)])
        inn = np.concatenate([[3], 4 + rs.choice(n_utt - 4, 11, replace=False)])
        picks.append((ic, inn))
    st = synth.make_state(52, 1)
    runs = {}
    for mode in ("padded", "store"):
        mk = store.collate if mode == "padded" else store.batch_index
        batches = [(mk(ic, T=40), mk(inn, T=40, with_labels=False)) for ic, inn in picks]
        if mode == "store":
            assert isinstance(batches[0][0]["net_input"]["feats"], D.StoreFeats)
        for ahead in (False, True):
            runs[(mode, ahead)] = _chain(cfg, precision, batches, st, ahead=ahead)
    _, _, prepped = runs[("store", True)]
    assert prepped == [False] + [True] * (K - 1), prepped
    want, want_losses, _ = runs[("padded", False)]
    for key in (("store", False), ("store", True), ("padded", True)):
        got, got_losses, _ = runs[key]
        for name, a, b in zip(("student", "teacher", "exp_avg", "exp_avg_sq", "dacp", "grad"), got, want):
            assert torch.equal(a, b), "%s: %s differs (max %.3g)" % (key, name, float((a - b).abs().max()))
        assert got_losses == want_losses, key


@pytest.mark.parametrize("precision,B,T,parts", [("fp16", 16, 40, 1), ("fp16", 16, 40, 2), ("fp16", 16, 40, 3),
                                                 ("fp16", 64, 300, 1), ("bf16", 64, 300, 3)])
def test_prefetch_under_exchange_equals_plain_chain(precision, B, T, parts):
    """The data-parallel layout (DADStep.prep_under_exchange, C ABI dad_step_backward_ahead_split +
    dad_step_prepare_rows): the deferred parts of the next batch's rows (1 clean: the weight gradient
    runs without its conversion; 2 noisy: the tail launch without its preparation; 3 both) are
    prepared on a second stream from the end of the backward on (under the all-reduce at N > 1; here
    on one GPU without one), the next step's encoder waiting on its event.  The chain equals the plain chain bit for bit, with the
    same steps skipping their own preparation as the tail-launch layout."""
    cfg = dad_oracle.make_cfg("iemocap")
    Bn, Tn = (12, 50) if B == 16 else (B, T)
    batches = [_device_batches(_problem(B=B, T=T, seed=61 + i, Bn=Bn, Tn=Tn))[:2] for i in range(3)]
    st = synth.make_state(61, 1)
    want, want_losses, _ = _chain(cfg, precision, batches, st, ahead=False)
    got, got_losses, prepped = _chain(cfg, precision, batches, st, ahead=True, wrong_at=3, split=parts)
    assert prepped == [False, True, True, True, False, True, True], prepped
    for name, a, b in zip(("student", "teacher", "exp_avg", "exp_avg_sq", "dacp", "grad"), got, want):
        assert torch.equal(a, b), "%s differs (max %.3g)" % (name, float((a - b).abs().max()))
    assert got_losses == want_losses


def test_prepare_rows_matches_step_preparation():
    """dad_step_prepare_rows writes exactly the prepared set a step's own preparation writes: a step
    run after it with cfg.prepped = 1 (rows taken from the set) equals the same step preparing its
    rows itself, bit for bit."""
    import ctypes
    import dadpkg
    PKG = dadpkg.pkg()
    L = PKG._lib.lib()
    cfg = dad_oracle.make_cfg("iemocap")
    c, n = _device_batches(_problem(B=16, T=40, seed=71, Bn=12, Tn=50))[:2]
    st = synth.make_state(71, 1)
    res = []
    for external in (False, True):
        step = gh.make_step(cfg, precision="fp16", rng="counter", seed=5)
        gh.load_state(step, st)
        if external:
            dcfg, bt, keep = step._batch_structs(c, n, 60, None, None)
            ws = step._workspace(dcfg)
            rc = L.dad_step_prepare_rows(dcfg, bt, PKG._lib.ptr(ws), step._stream(),
                                         PKG._lib.PREP_CLEAN | PKG._lib.PREP_NOISY)
            assert rc == 0
            step._prepped_key = step._prep_key(dcfg, bt)      # as if the previous step had prepared it
        out = step.step(c, n, 60)
        assert step.last_prepped == external
        torch.cuda.synchronize()
        res.append((_state(step), {k: float(v) for k, v in out.items()}))
    for name, a, b in zip(("student", "teacher", "exp_avg", "exp_avg_sq", "dacp", "grad"), res[1][0], res[0][0]):
        assert torch.equal(a, b), name
    assert res[0][1] == res[1][1]
    # FP32 has no prepared rows; bad part masks are refused
    dcfg, bt, _ = step._batch_structs(c, n, 60, None, None)
    ws = step._workspace(dcfg)
    assert L.dad_step_prepare_rows(dcfg, bt, PKG._lib.ptr(ws), step._stream(), 4) == 1001
    dcfg.precision = PKG._lib.PREC_FP32
    assert L.dad_step_prepare_rows(dcfg, bt, PKG._lib.ptr(ws), step._stream(), 3) == 1004


def test_timing_reset_counts_only_later_steps():
    """dad_timing_reset (ABI 7, bench.py's warm-up): the steps before the reset are not counted and
    the session's events stay usable: every step timed (every = 1), 3 steps, reset, 2 steps -> the
    encoder's count is 2 and its mean a positive duration; a reset with no session is refused."""
    import dadpkg
    L = dadpkg.pkg()._lib
    cfg = dad_oracle.make_cfg("iemocap")
    st = synth.make_state(3, 1, tau_range=(0.0, 0.01))
    batches = [_device_batches(_problem(B=16, T=40, seed=41 + i))[:2] for i in range(2)]
    step = gh.make_step(cfg, precision="fp16", rng="counter", seed=5)
    gh.load_state(step, st)
    timer = L.KernelTimer(1, 8)
    try:
        for k in range(3):
            step.step(*batches[k % len(batches)], 60)
        torch.cuda.synchronize()
        timer.reset()
        for k in range(2):
            step.step(*batches[k % len(batches)], 60)
        torch.cuda.synchronize()
    finally:
        res = timer.stop()
    ms, n = res["encode"]
    assert n == 2 and ms > 0.0, res
    with pytest.raises(L.DadError):
        L.KernelTimer.reset(timer)   # (stopped: no active session)
