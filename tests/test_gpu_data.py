"""Device-resident data path on the MI355X: the dad_collate gather (csrc/collate.hip, through
the C ABI) against the reference loaders' golden outputs and the NumPy oracle.  Bit-exact:
collation copies and widens, it does not round."""
import ctypes

import numpy as np
import pytest
import torch

import dadpkg
import gpu_harness as gh
from oracle import dad_oracle, synth
from oracle import data_oracle as do
from test_data_cpu import CASIA_LOADERS, IEMOCAP_LOADERS, _golden

pytestmark = pytest.mark.gpu
PKG = dadpkg.pkg()
D = PKG.data


def _compare(g, name, loader, seed, with_ids=True):
    torch.manual_seed(seed)
    shapes, pads, labs, sums, sumsqs, ids = [], [], [], [], [], []
    for batch in loader:
        x = batch["net_input"]["feats"].cpu().numpy().astype(np.float64)
        shapes.append(x.shape[:2])
        pads.append(batch["net_input"]["padding_mask"].cpu().numpy().reshape(-1))
        lab = batch.get("labels")
        labs.append(np.full(x.shape[0], -2, np.int64) if lab is None else lab.cpu().numpy())
        sums.append(x.sum())
        sumsqs.append((x * x).sum())
        if with_ids:
            ids.append(batch["id"].cpu().numpy())
    np.testing.assert_array_equal(np.array(shapes), g[name + "_shapes"], err_msg=name)
    np.testing.assert_array_equal(np.concatenate(pads), g[name + "_pad"], err_msg=name)
    np.testing.assert_array_equal(np.concatenate(labs), g[name + "_labels"], err_msg=name)
    np.testing.assert_array_equal(np.array(sums), g[name + "_sum"], err_msg=name)
    np.testing.assert_array_equal(np.array(sumsqs), g[name + "_sumsq"], err_msg=name)
    if with_ids:
        np.testing.assert_array_equal(np.concatenate(ids), g[name + "_ids"], err_msg=name)


def test_iemocap_device_loaders_match_reference(tmp_path):
    g = _golden("data_iemocap")
    seed, bs, fold = int(g["seed"]), int(g["batch_size"]), int(g["fold"])
    do.write_synthetic_split(str(tmp_path), seed, n_utt=150, max_len=40, flavor="iemocap")
    noisy = D.get_cv_dataloaders_noisy(str(tmp_path), bs, fold_id=fold)
    clean = D.get_cv_dataloaders(str(tmp_path), bs, fold_id=fold)[:3]
    for (name, _, _, _, s), ld in zip(IEMOCAP_LOADERS, list(noisy) + list(clean)):
        _compare(g, name, ld, s)


def test_casia_device_loaders_match_reference(tmp_path):
    g = _golden("data_casia")
    seed, bs, fold = int(g["seed"]), int(g["batch_size"]), int(g["fold"])
    prefix = do.write_synthetic_split(str(tmp_path), seed, n_utt=90, max_len=30, flavor="casia")
    np.random.seed(seed)
    store, spk = D.load_casia_noisy_data(prefix)
    loaders = D.create_casia_noisy_speaker_isolated_loaders(store, spk, fold, bs)
    for (name, _, _, _, s), ld in zip(CASIA_LOADERS, loaders):
        _compare(g, name, ld, s, with_ids=False)


def test_emodb_device_loaders_match_reference(tmp_path):
    g = _golden("data_emodb")
    seed, bs, fold = int(g["seed"]), int(g["batch_size"]), int(g["fold"])
    prefix = do.write_synthetic_split(str(tmp_path), seed, n_utt=160, max_len=30, flavor="emodb")
    np.random.seed(seed)
    store, spk = D.load_emodb_noisy_data(prefix)
    loaders = D.create_emodb_noisy_speaker_isolated_loaders(store, spk, fold, bs)
    for (name, _, _, _, s), ld in zip(CASIA_LOADERS, loaders):
        _compare(g, name, ld, s, with_ids=False)


def _store(seed, n, max_len, dtype=torch.float32):
    rs = np.random.RandomState(seed)
    sizes = rs.randint(1, max_len + 1, size=n)
    feats = rs.standard_normal((int(sizes.sum()), 768)).astype(np.float32)
    offsets = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    labels = rs.randint(0, 4, size=n)
    return feats, sizes, offsets, labels, D.FeatureStore(feats, sizes, offsets, labels, dtype=dtype)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
def test_collate_matches_oracle_each_store_dtype(dtype):
    feats, sizes, offsets, labels, st = _store(21, 40, 33, dtype)
    # the oracle gathers the store's values widened to f32 (Tensor.float())
    ref_feats = torch.from_numpy(feats).to(dtype).float().numpy()
    for index in ([3], [0, 1, 2, 3], list(range(39, -1, -3)), [7, 7, 7]):
        got = st.collate(index)
        ref = do.collate(ref_feats, sizes, offsets, labels, index)
        np.testing.assert_array_equal(got["net_input"]["feats"].cpu().numpy(), ref["feats"])
        np.testing.assert_array_equal(got["net_input"]["padding_mask"].cpu().numpy(), ref["padding_mask"])
        np.testing.assert_array_equal(got["labels"].cpu().numpy(), ref["labels"])
        np.testing.assert_array_equal(got["id"].cpu().numpy(), ref["id"])


def test_collate_explicit_pad_length_and_unlabeled():
    feats, sizes, offsets, labels, st = _store(22, 12, 9)
    index = [4, 0, 11]
    T = int(sizes[index].max()) + 5          # longer than the batch max: extra rows are padding
    got = st.collate(index, T=T, with_labels=False)
    ref = do.collate(feats, sizes, offsets, None, index)
    x = got["net_input"]["feats"].cpu().numpy()
    np.testing.assert_array_equal(x[:, :ref["feats"].shape[1]], ref["feats"])
    assert not x[:, ref["feats"].shape[1]:].any()
    assert got["net_input"]["padding_mask"].cpu().numpy()[:, ref["feats"].shape[1]:].all()
    assert got["labels"] is None


def test_collate_c_abi_out_of_range_index_is_padding():
    feats, sizes, offsets, labels, st = _store(23, 10, 6)
    L = PKG.lib()
    index = torch.tensor([2, -1, 10, 5], dtype=torch.int64, device="cuda")
    B, T = 4, 6
    out = torch.full((B, T, 768), 7.0, device="cuda")
    pad = torch.full((B, T), 9, dtype=torch.uint8, device="cuda")
    lab = torch.full((B,), 9, dtype=torch.int64, device="cuda")
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    rc = L.dad_collate(p(st.feats), 0, p(st.offsets_d), p(st.sizes_d), len(st), p(index), B, T, p(out), p(pad),
                       p(st.labels_d), p(lab), torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    x, m, y = out.cpu().numpy(), pad.cpu().numpy(), lab.cpu().numpy()
    for i in (1, 2):
        assert not x[i].any() and m[i].all() and y[i] == -1
    ref = do.collate(feats, sizes, offsets, labels, [2, 5])
    for i, j in ((0, 0), (3, 1)):
        n = ref["feats"].shape[1]
        np.testing.assert_array_equal(x[i, :n], ref["feats"][j])
        assert not x[i, n:].any()
        np.testing.assert_array_equal(m[i, :n], ref["padding_mask"][j])
        assert m[i, n:].all() and y[i] == labels[[2, 5][j]]
    # argument errors come back as codes, nothing is launched
    assert L.dad_collate(None, 0, p(st.offsets_d), p(st.sizes_d), 10, p(index), B, T, p(out), p(pad), None, None,
                         None) == 1001
    assert L.dad_collate(p(st.feats), 5, p(st.offsets_d), p(st.sizes_d), 10, p(index), B, T, p(out), p(pad), None,
                         None, None) == 1001
    assert L.dad_collate(p(st.feats), 0, p(st.offsets_d), p(st.sizes_d), 10, p(index), 0, T, p(out), p(pad), None,
                         None, None) == 1002


def test_collate_bench_shape_bit_exact():
    """The benchmark's shape: B=64, T=300 from a store of 160 utterances up to 300 frames."""
    rs = np.random.RandomState(24)
    sizes = rs.randint(200, 301, size=160)
    sizes[rs.choice(160, 8, replace=False)] = 300
    feats = rs.standard_normal((int(sizes.sum()), 768)).astype(np.float32)
    offsets = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    st = D.FeatureStore(feats, sizes, offsets, rs.randint(0, 4, size=160))
    index = rs.permutation(160)[:64]
    index[0] = int(np.argmax(sizes))
    got = st.collate(index)
    ref = do.collate(feats, sizes, offsets, st.labels, index)
    assert got["net_input"]["feats"].shape == (64, 300, 768)
    np.testing.assert_array_equal(got["net_input"]["feats"].cpu().numpy(), ref["feats"])
    np.testing.assert_array_equal(got["net_input"]["padding_mask"].cpu().numpy(), ref["padding_mask"])


def _step_outputs(step, clean, noisy, epoch, draws, Bc, Bn):
    losses = step.step(clean, noisy, epoch, draws=draws)
    torch.cuda.synchronize()
    out = {k: v.detach().cpu().numpy() for k, v in step.outputs(Bc, Bn).items() if torch.is_tensor(v)}
    out.update({k: np.float32(float(v)) for k, v in losses.items()})
    out["student"] = step.model.student_flat.detach().cpu().numpy()
    out["teacher"] = step.model.teacher_flat.detach().cpu().numpy()
    out["dacp"] = step.dacp.cpu().numpy()
    return out


@pytest.mark.parametrize("precision,rng", [("fp32", "explicit"), ("bf16", "explicit"), ("bf16", "counter"),
                                           ("fp16", "explicit"), ("fp16", "counter")])
def test_store_mode_step_equals_padded_step(precision, rng):
    """Store mode (the encoder gathers rows straight from the FeatureStore, no padded copy)
    computes exactly what the padded batch computes: same losses, logits, embeddings, updated
    student/teacher and DACP state, bit for bit (padding frames are masked everywhere)."""
    cfg = dad_oracle.make_cfg("iemocap")
    rs = np.random.RandomState(40)
    sizes = rs.randint(5, 38, size=48)
    feats = rs.standard_normal((int(sizes.sum()), 768)).astype(np.float32) * 0.5
    offsets = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    st = D.FeatureStore(feats, sizes, offsets, rs.randint(0, 4, size=48))
    ic, inn = rs.choice(48, 12, replace=False), rs.choice(48, 10, replace=False)
    Tc, Tn = int(sizes[ic].max()), int(sizes[inn].max())
    draws = None
    if rng == "explicit":
        draws = {"nw": rs.standard_normal((10, Tn, 768)).astype(np.float32),
                 "ns": rs.standard_normal((10, Tn, 768)).astype(np.float32),
                 "u": rs.rand(768).astype(np.float32), "start": rs.randint(0, max(1, Tn - 4), size=10),
                 "keep1": rs.rand(12, 256) > 0.1, "keep2": rs.rand(10, 256) > 0.1}
    state = synth.make_state(40, 1)
    outs = []
    for mode in ("padded", "store"):
        step = gh.make_step(cfg, precision=precision, rng=rng, seed=9)
        gh.load_state(step, state)
        mk = st.collate if mode == "padded" else st.batch_index
        clean, noisy = mk(ic), mk(inn, with_labels=False)
        if mode == "store":
            assert isinstance(clean["net_input"]["feats"], D.StoreFeats)
        outs.append(_step_outputs(step, clean, noisy, 60, draws, 12, 10))
    a, b = outs
    assert set(a) == set(b)
    for k in a:
        np.testing.assert_array_equal(b[k], a[k], err_msg=k)


@pytest.mark.parametrize("precision", ["bf16", "fp16"])
def test_device_batches_drive_the_step(tmp_path, precision):
    """The loaders' batches go straight into DADStep (the reference loop body); fused loaders
    (store mode) give the same training trajectory as collating loaders (bf16 and the timed fp16
    mode)."""
    do.write_synthetic_split(str(tmp_path), 31, n_utt=80, max_len=25, flavor="iemocap")
    res = []
    for fused in (False, True):
        clean = D.get_cv_dataloaders(str(tmp_path), 8, fold_id=1)[0]
        noisy = D.get_cv_dataloaders_noisy(str(tmp_path), 8, fold_id=1)[0]
        clean.fused = noisy.fused = fused
        torch.manual_seed(1)
        model = PKG.SSRLModel().cuda()
        step = PKG.DADStep(model, flavor="iemocap", precision=precision, rng="counter", seed=2)
        torch.manual_seed(0)
        ci, ni = iter(clean), iter(noisy)
        for _ in range(3):
            losses = step.step(next(ci), next(ni), 60)
        torch.cuda.synchronize()
        assert all(np.isfinite(float(v)) for v in losses.values())
        res.append((np.array([float(v) for v in losses.values()]), model.student_flat.detach().cpu().numpy()))
    np.testing.assert_array_equal(res[0][0], res[1][0])
    np.testing.assert_array_equal(res[0][1], res[1][1])


@pytest.mark.parametrize("with_labels,style", [(True, "iemocap"), (False, "casia")])
def test_fused_loader_epoch_views_equal_batch_index(with_labels, style):
    """Store-mode loaders prepare an epoch's rows, lengths, masks and labels at its first next() and
    hand out views (data._DeviceLoaderIter._epoch_index): every batch of two epochs (ragged last
    batch, batch-dependent T) equals FeatureStore.batch_index on the same indices."""
    rs = np.random.RandomState(44)
    sizes = rs.randint(1, 41, size=37)
    feats = rs.standard_normal((int(sizes.sum()), 768)).astype(np.float32)
    offsets = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    st = D.FeatureStore(feats, sizes, offsets, rs.randint(0, 4, size=37))
    g = torch.Generator()
    g.manual_seed(5)
    L = D.DeviceLoader(st, batch_size=8, shuffle=True, generator=g, style=style, with_labels=with_labels, fused=True)
    for _ in range(2):
        n = 0
        for batch in L:
            f = batch["net_input"]["feats"]
            assert isinstance(f, D.StoreFeats)
            want = st.batch_index(f.index, style=style, with_labels=with_labels)
            wf = want["net_input"]["feats"]
            assert f.shape == wf.shape
            for a, b in ((f.rows, wf.rows), (f.lens, wf.lens), (f.index_d, wf.index_d),
                         (batch["net_input"]["padding_mask"], want["net_input"]["padding_mask"])):
                assert a.dtype == b.dtype and torch.equal(a, b)
            assert set(batch) == set(want)
            if "labels" in want and want["labels"] is not None:
                assert torch.equal(batch["labels"], want["labels"])
            if "id" in want:
                assert torch.equal(batch["id"], want["id"])
            n += len(f.index)
        assert n == 37
