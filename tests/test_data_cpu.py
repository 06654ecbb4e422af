"""Data path on the CPU: the oracle restatement against the reference's own loaders (golden
fixtures tests/golden/data_*.npz from tests/golden/gen_data_golden.py), and the product's
host-side logic (file parsing, fold splits, the sampler's batch order) against the oracle.
The device gather itself is tested in test_gpu_data.py."""
import os

import numpy as np
import pytest
import torch

from oracle import data_oracle as do
import dadpkg

PKG = dadpkg.pkg()

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
IEMOCAP_LOADERS = [("noisy_student", "train", True, False, 100), ("noisy_teacher", "train", True, False, 101),
                   ("noisy_val", "val", False, True, 102), ("noisy_test", "test", False, True, 103),
                   ("clean_train", "train", True, True, 200), ("clean_val", "val", False, True, 201),
                   ("clean_test", "test", False, True, 202)]
CASIA_LOADERS = [("noisy_student", "train", True, False, 300), ("noisy_teacher", "train", True, False, 301),
                 ("noisy_val", "val", False, True, 302), ("noisy_test", "test", False, True, 303)]


def _golden(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz")))


def _torch_batches(n, bs, shuffle, seed):
    """The reference DataLoader's index stream: torch.manual_seed(seed), then iterate."""
    torch.manual_seed(seed)
    dl = torch.utils.data.DataLoader(range(n), batch_size=bs, shuffle=shuffle, collate_fn=lambda b: b)
    return [np.asarray(b, np.int64) for b in dl]


def _check_loader(g, name, sub, batches, style_ids=True):
    feats, sizes, offsets, labels = sub
    shapes, pads, labs, sums, sumsqs, ids = [], [], [], [], [], []
    for b in batches:
        c = do.collate(feats, sizes, offsets, labels, b)
        x = c["feats"].astype(np.float64)
        shapes.append(c["feats"].shape[:2])
        pads.append(c["padding_mask"].reshape(-1))
        labs.append(np.full(len(b), -2, np.int64) if c["labels"] is None else c["labels"])
        sums.append(x.sum())
        sumsqs.append((x * x).sum())
        ids.append(c["id"])
    np.testing.assert_array_equal(np.array(shapes), g[name + "_shapes"], err_msg=name)
    np.testing.assert_array_equal(np.concatenate(pads), g[name + "_pad"], err_msg=name)
    np.testing.assert_array_equal(np.concatenate(labs), g[name + "_labels"], err_msg=name)
    np.testing.assert_array_equal(np.array(sums), g[name + "_sum"], err_msg=name)
    np.testing.assert_array_equal(np.array(sumsqs), g[name + "_sumsq"], err_msg=name)
    if style_ids:
        np.testing.assert_array_equal(np.concatenate(ids), g[name + "_ids"], err_msg=name)


def test_oracle_iemocap_loaders_match_reference(tmp_path):
    g = _golden("data_iemocap")
    seed, bs, fold = int(g["seed"]), int(g["batch_size"]), int(g["fold"])
    prefix = do.write_synthetic_split(str(tmp_path), seed, n_utt=150, max_len=40, flavor="iemocap")
    _, sizes, offsets, labs = do.load_emotion2vec_dataset(prefix, min_length=3, max_length=30)
    np.testing.assert_array_equal(sizes, g["parse_sizes"])
    np.testing.assert_array_equal(offsets, g["parse_offsets"])
    assert list(labs) == list(g["parse_labels"])
    np.testing.assert_array_equal(do.get_session_ids(prefix, 150), g["session_ids"])
    d = do.load_ssl_features(str(tmp_path))
    splits = dict(zip(("train", "val", "test"), do.session_split(d["session_ids"], fold)))
    for name, part, shuffle, labeled, s in IEMOCAP_LOADERS:
        idx = splits[part]
        sub = do.make_subset(d["feats"], d["sizes"], d["offsets"], d["labels"] if labeled else None, idx)
        _check_loader(g, name, sub, _torch_batches(len(idx), bs, shuffle, s))


def test_oracle_casia_loaders_match_reference(tmp_path):
    g = _golden("data_casia")
    seed, bs, fold = int(g["seed"]), int(g["batch_size"]), int(g["fold"])
    prefix = do.write_synthetic_split(str(tmp_path), seed, n_utt=90, max_len=30, flavor="casia")
    np.random.seed(seed)
    d = do.load_casia_noisy_data(prefix)
    tr, va, te = do.casia_speaker_split(d["speakers"], fold)
    splits = {"train": tr, "val": va, "test": te}
    for name, part, shuffle, labeled, s in CASIA_LOADERS:
        idx = splits[part]
        sub = do.make_subset(d["feats"], d["sizes"], d["offsets"], d["labels"] if labeled else None, idx)
        _check_loader(g, name, sub, _torch_batches(len(idx), bs, shuffle, s), style_ids=False)


def test_oracle_emodb_loaders_match_reference(tmp_path):
    g = _golden("data_emodb")
    seed, bs, fold = int(g["seed"]), int(g["batch_size"]), int(g["fold"])
    prefix = do.write_synthetic_split(str(tmp_path), seed, n_utt=160, max_len=30, flavor="emodb")
    np.random.seed(seed)
    d = do.load_casia_noisy_data(prefix)            # E/ reads the same four files
    tr, va, te = do.emodb_speaker_split(d["speakers"], fold)
    splits = {"train": tr, "val": va, "test": te}
    for name, part, shuffle, labeled, s in CASIA_LOADERS:
        idx = splits[part]
        sub = do.make_subset(d["feats"], d["sizes"], d["offsets"], d["labels"] if labeled else None, idx)
        _check_loader(g, name, sub, _torch_batches(len(idx), bs, shuffle, s), style_ids=False)


def test_product_emodb_folds_match_oracle():
    for f in range(10):
        assert PKG.data.get_emodb_fold_speakers(f)[1:] == (do.EMODB_SPEAKERS[(f + 1) % 10], do.EMODB_SPEAKERS[f])
    with pytest.raises(ValueError):
        PKG.data.get_emodb_fold_speakers(10)


def test_product_parsers_match_oracle(tmp_path):
    D = PKG.data
    prefix = do.write_synthetic_split(str(tmp_path), 9, n_utt=60, max_len=12, flavor="iemocap")
    for kw in (dict(min_length=3, max_length=None), dict(min_length=1, max_length=8), dict(ignore_labels=True)):
        a = D.load_emotion2vec_dataset(prefix, **kw)
        b = do.load_emotion2vec_dataset(prefix, **kw)
        np.testing.assert_array_equal(np.asarray(a[0]), b[0])
        np.testing.assert_array_equal(a[1], b[1])
        np.testing.assert_array_equal(a[2], b[2])
        assert a[3] == b[3]
    assert D.get_session_ids(prefix, 60) == do.get_session_ids(prefix, 60)
    assert D.get_session_ids(str(tmp_path / "missing"), 3) == [None] * 3
    for f in range(1, 6):
        assert D.get_fold_sessions(f) == do.get_fold_sessions(f)
    with pytest.raises(ValueError):
        D.get_fold_sessions(0)


class _HostStore:
    """Stand-in for FeatureStore on the CPU: records what the loader asks to collate."""

    def __init__(self, sizes, labels=None):
        self.sizes = np.asarray(sizes, np.int64)
        self.labels = labels
        self.device = torch.device("cpu")
        self.calls = []

    def __len__(self):
        return len(self.sizes)

    def collate(self, index, index_d=None, T=None, style="iemocap", with_labels=True):
        self.calls.append((np.asarray(index).copy(), index_d.numpy().copy(), T, style, with_labels))
        return index


@pytest.mark.parametrize("shuffle,drop_last", [(True, False), (False, False), (True, True)])
def test_device_loader_batch_order_matches_torch_dataloader(shuffle, drop_last):
    sizes = np.random.RandomState(3).randint(1, 50, size=37)
    st = _HostStore(sizes, labels=np.zeros(37))
    L = PKG.data.DeviceLoader(st, batch_size=8, shuffle=shuffle, drop_last=drop_last)
    torch.manual_seed(11)
    got = list(L)
    torch.manual_seed(11)
    ref = [np.asarray(b) for b in torch.utils.data.DataLoader(range(37), batch_size=8, shuffle=shuffle,
                                                              drop_last=drop_last, collate_fn=lambda b: b)]
    assert len(got) == len(ref) == len(L)
    for g, r, call in zip(got, ref, st.calls):
        np.testing.assert_array_equal(g, r)
        np.testing.assert_array_equal(call[1], r)           # the device index slice is the batch
        assert call[2] == sizes[r].max()                     # padded length = the batch max size


@pytest.mark.parametrize("with_generator", [False, True])
def test_device_loader_epochs_and_rng_state_match_torch_dataloader(with_generator):
    """Two epochs of a shuffled DeviceLoader (its batch order drawn without the DataLoader's
    per-index iteration) against torch's DataLoader: the same batches in both epochs and the same
    global (and generator) RNG state afterwards."""
    sizes = np.full(50, 4)
    st = _HostStore(sizes, labels=np.zeros(50))
    gen = (lambda: torch.Generator().manual_seed(9)) if with_generator else (lambda: None)
    L = PKG.data.DeviceLoader(st, batch_size=7, shuffle=True, generator=gen())
    torch.manual_seed(21)
    got = [list(L), list(L)]
    after = torch.rand(3)
    ref_loader = torch.utils.data.DataLoader(range(50), batch_size=7, shuffle=True, generator=gen(),
                                             collate_fn=lambda b: b)
    torch.manual_seed(21)
    ref = [[np.asarray(b) for b in ref_loader], [np.asarray(b) for b in ref_loader]]
    assert torch.equal(after, torch.rand(3))
    for ge, re in zip(got, ref):
        assert len(ge) == len(re)
        for g, r in zip(ge, re):
            np.testing.assert_array_equal(g, r)


def test_device_loader_draws_rng_like_the_reference_loop():
    """iter(a), iter(b), next(a), next(b) -- the reference's epoch start (I/train.py:479-483):
    each loader must take its sampler seed at its first next(), not at iter()."""
    n, bs = 30, 7
    sa, sb = _HostStore(np.full(n, 5)), _HostStore(np.full(n, 5))
    A, B = PKG.data.DeviceLoader(sa, bs, shuffle=True), PKG.data.DeviceLoader(sb, bs, shuffle=True)
    torch.manual_seed(5)
    ia, ib = iter(A), iter(B)
    a0, b0 = next(ia), next(ib)
    torch.manual_seed(5)
    mk = lambda: torch.utils.data.DataLoader(range(n), batch_size=bs, shuffle=True, collate_fn=lambda b: b)
    ra, rb = iter(mk()), iter(mk())
    np.testing.assert_array_equal(a0, next(ra))
    np.testing.assert_array_equal(b0, next(rb))
    np.testing.assert_array_equal(next(ia), next(ra))
