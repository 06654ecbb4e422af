"""Epoch-level state on the MI355X (checkpoint.py): a run resumed from a checkpoint continues
bit for bit like the uninterrupted run, and train_epoch drives the device loaders through the
fused step with the DACP epoch-end update."""
import numpy as np
import pytest
import torch

import dadpkg
import gpu_harness as gh
from oracle import dad_oracle, synth
from oracle import data_oracle as do

pytestmark = pytest.mark.gpu
PKG = dadpkg.pkg()
CK = PKG.checkpoint


def _batches(seed, k):
    rs = np.random.RandomState(seed)
    sizes = rs.randint(8, 40, size=64)
    feats = rs.standard_normal((int(sizes.sum()), 768)).astype(np.float32)
    offsets = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    st = PKG.data.FeatureStore(feats, sizes, offsets, rs.randint(0, 4, size=64))
    return [(st.collate(rs.choice(64, 12, replace=False)), st.collate(rs.choice(64, 10, replace=False), with_labels=False))
            for _ in range(k)]


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_resume_from_checkpoint_is_bit_exact(tmp_path, precision):
    cfg = dad_oracle.make_cfg("iemocap")
    data = _batches(50, 4)
    state = synth.make_state(50, 1)
    a = gh.make_step(cfg, precision=precision, rng="counter", seed=4)
    gh.load_state(a, state)
    for i in range(2):
        a.step(*data[i], 60)
    path = str(tmp_path / "ck.pth")
    CK.save_checkpoint(path, 60, a.model, a, clean_results={"confusion_matrix": np.eye(4, dtype=np.int64)})
    b = gh.make_step(cfg, precision=precision, rng="counter", seed=4)
    CK.load_checkpoint(path, b.model, b)
    for i in range(2, 4):
        la, lb = a.step(*data[i], 60), b.step(*data[i], 60)
    torch.cuda.synchronize()
    for k in la:
        assert float(la[k]) == float(lb[k]), k
    for x, y in ((a.model.student_flat, b.model.student_flat), (a.model.teacher_flat, b.model.teacher_flat),
                 (a.exp_avg, b.exp_avg), (a.exp_avg_sq, b.exp_avg_sq), (a.dacp, b.dacp)):
        assert torch.equal(x, y)
    assert a.adam_step == b.adam_step == int(state["nstep"]) + 4


def test_train_epoch_runs_loaders_and_epoch_end(tmp_path):
    do.write_synthetic_split(str(tmp_path), 61, n_utt=90, max_len=30, flavor="iemocap")
    clean = PKG.data.get_cv_dataloaders(str(tmp_path), 8, fold_id=2)[0]
    noisy = PKG.data.get_cv_dataloaders_noisy(str(tmp_path), 8, fold_id=2)[0]
    torch.manual_seed(0)
    model = PKG.SSRLModel().cuda()
    step = PKG.DADStep(model, flavor="iemocap", precision="bf16", rng="counter", seed=1)
    q0 = step.class_quality_scores.clone()
    avg = CK.train_epoch(step, clean, noisy, 40)
    assert set(avg) >= {"total_loss", "supervised_ce_loss", "consistency_loss", "ecda_loss", "range_flag"}
    assert avg["range_flag"] == 0
    assert all(np.isfinite(v) for v in avg.values())
    assert step.adam_step == min(len(clean), len(noisy))
    assert not torch.equal(step.class_quality_scores, q0)   # DACP quality updated at epoch end
    warm = CK.train_epoch(step, clean, noisy, 3)              # warm-up: no epoch-end update
    assert np.isfinite(warm["total_loss"])


def _store_batches(seed, k, length=30, mode="batch_index"):
    """Batches of equal-length utterances from a data.FeatureStore, so consecutive batches share
    their geometry and the next batch's rows can be prepared ahead: store mode (batch_index: rows
    gathered from the store) or padded copies (collate)."""
    rs = np.random.RandomState(seed)
    sizes = np.full(64, length)
    feats = rs.standard_normal((int(sizes.sum()), 768)).astype(np.float32)
    offsets = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    st = PKG.data.FeatureStore(feats, sizes, offsets, rs.randint(0, 4, size=64))
    f = getattr(st, mode)
    return [(f(rs.choice(64, 12, replace=False)), f(rs.choice(64, 10, replace=False), with_labels=False))
            for _ in range(k)]


@pytest.mark.parametrize("mode", ["batch_index", "collate"])
def test_store_mode_prefetch_chain_is_bit_exact(mode):
    """Store-mode batches (rows gathered from the feature store through dad_batch.rowc..lenn) with
    the next batch prepared in each tail launch: the same parameters, moments, DACP state and
    losses as the chain that prepares every batch itself (fp16)."""
    cfg = dad_oracle.make_cfg("iemocap")
    data = _store_batches(51, 5, mode=mode)
    state = synth.make_state(51, 1)
    runs = []
    for ahead in (False, True):
        s = gh.make_step(cfg, precision="fp16", rng="counter", seed=6)
        gh.load_state(s, state)
        flags = []
        for i in range(len(data)):
            nxt = data[i + 1] if ahead and i + 1 < len(data) else None
            l = s.step(*data[i], 60, next_batch=nxt)
            flags.append(s.last_prepped)
        torch.cuda.synchronize()
        runs.append((s, {k: float(v) for k, v in l.items()}, flags))
    (a, la, fa), (b, lb, fb) = runs
    assert fa == [False] * 5 and fb == [False, True, True, True, True]
    assert la == lb
    for x, y in ((a.model.student_flat, b.model.student_flat), (a.model.teacher_flat, b.model.teacher_flat),
                 (a.exp_avg, b.exp_avg), (a.exp_avg_sq, b.exp_avg_sq), (a.dacp, b.dacp)):
        assert torch.equal(x, y)


def test_host_next_batch_is_not_prepared_ahead():
    """a next batch of host tensors is not prepared ahead (it would be copied here and
    again by the step that runs it, and the rows prepared from the first copy would not match);
    the same batch on the device is."""
    cfg = dad_oracle.make_cfg("iemocap")
    from test_gpu_parity import _problem
    from test_gpu_graph import _device_batches
    host = gh.batches(_problem(B=12, T=40, seed=71, Bn=10, Tn=44))[:2]
    dev = _device_batches(_problem(B=12, T=40, seed=72, Bn=10, Tn=44))[:2]
    s = gh.make_step(cfg, precision="fp16", rng="counter", seed=7)
    gh.load_state(s, synth.make_state(71, 1))
    s.step(dev[0], dev[1], 60, next_batch=host)
    assert s._prepped_key is None
    s.step(host[0], host[1], 60, next_batch=dev)
    assert not s.last_prepped and s._prepped_key is not None
    s.step(dev[0], dev[1], 60)
    torch.cuda.synchronize()
    assert s.last_prepped
