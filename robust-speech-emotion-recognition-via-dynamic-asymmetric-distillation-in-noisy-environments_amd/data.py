"""Device-resident data path: the feature store in HBM and collation as a device gather.

Mirrors the reference's loader surface so a trainer can swap its
DataLoaders for these without touching the loop:

  load_emotion2vec_dataset, get_session_ids, get_fold_sessions     I/dataload_noisy.py:17-90
  get_cv_dataloaders (clean)                                        I/dataload_clean.py:222-293
  get_cv_dataloaders_noisy                                          I/dataload_noisy.py:159-231
  load_casia_noisy_data, create_casia_noisy_speaker_isolated_loaders C/dataload_casia_noisy.py:109-292
  load_emodb_noisy_data, create_emodb_noisy_speaker_isolated_loaders E/dataload_emodb_noisy.py:20-345

What changes is where the bytes live.  The reference slices each sample out of a host NumPy
array, widens it to f32 and pads the batch in a Python loop (I/dataload_noisy.py:104-129),
then the trainer copies the batch to the device.  Here the whole split (IEMOCAP: ~5.5 k
utterances x ~225 frames x 768 f32 = 3.8 GB) is uploaded ONCE into a `FeatureStore`; a
fold subset is an index remap over the same store (the reference copies the subset's rows
into a new array, create_subset, I/dataload_noisy.py:193-205: same rows, same order); a
batch is a list of sample indices and `dad_collate` (csrc/collate.hip) gathers, widens and
pads it on the device.  Sampling order is the reference's: the index stream comes from a
torch DataLoader over sample indices with the same batch_size/shuffle, drained at the first
`next()` exactly when the reference's sampler draws its seed, so torch.manual_seed(k)
before an epoch gives the reference's batches.  One H2D copy of the epoch's index list per
epoch; nothing per step.
"""
import contextlib
import os

import numpy as np
import torch

from . import _lib

STORE_DTYPES = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}    # DAD_STORE_* (include/dad.h)
IEMOCAP_LABEL_DICT = {"ang": 0, "hap": 1, "neu": 2, "sad": 3}             # I/config.py:39-44
CASIA_LABEL_DICT = {"angry": 0, "happy": 1, "neutral": 2, "sad": 3}       # C/config_casia.py:42-47
_UPLOAD_CHUNK = 64 << 20


def _device(device):
    d = torch.device(device if device is not None else "cuda")
    if d.type != "cuda" or not torch.cuda.is_available():
        raise RuntimeError("the device-resident data path needs the MI355X (got device %s)" % d)
    # an explicit index: DADStep compares the store's device with its own ("cuda:0"), and a bare
    # "cuda" would compare unequal and send every store-mode batch through a padded copy
    return d if d.index is not None else torch.device("cuda", torch.cuda.current_device())


class FeatureStore:
    """All frames of one split resident in HBM: feats [frames][768] (f32, or f16/bf16 to halve
    the footprint; collation widens to f32 exactly as Tensor.float() does), per-sample
    offsets/sizes (int64/int32) and optional int64 labels, on the device and on the host (the
    host copy of sizes gives each batch's padded length without a device read)."""

    def __init__(self, feats, sizes, offsets, labels=None, device=None, dtype=None):
        dev = _device(device)
        sizes = np.asarray(sizes, dtype=np.int64).reshape(-1)
        offsets = np.asarray(offsets, dtype=np.int64).reshape(-1)
        if sizes.shape != offsets.shape:
            raise ValueError("sizes and offsets differ in length")
        if torch.is_tensor(feats):
            src_dtype = feats.dtype
        else:
            feats = np.asarray(feats) if not isinstance(feats, np.memmap) else feats
            src_dtype = {np.dtype(np.float32): torch.float32, np.dtype(np.float16): torch.float16}.get(feats.dtype)
            if src_dtype is None:
                feats = feats.astype(np.float32)
                src_dtype = torch.float32
        dtype = dtype or src_dtype
        if dtype not in STORE_DTYPES:
            raise ValueError("store dtype must be float32, float16 or bfloat16, got %s" % dtype)
        if feats.ndim != 2 or feats.shape[1] != 768:
            raise ValueError("feats must be [frames, 768], got %s" % (tuple(feats.shape),))
        if len(sizes) and (offsets.min() < 0 or (offsets + sizes).max() > feats.shape[0] or sizes.min() < 0):
            raise ValueError("a sample's [offset, offset + size) leaves the feature array")
        self.feats = torch.empty(feats.shape[0], 768, dtype=dtype, device=dev)
        step = max(1, _UPLOAD_CHUNK // (768 * 4))
        for r0 in range(0, feats.shape[0], step):    # chunked: a memory-mapped .npy never lands whole in RAM
            part = feats[r0:r0 + step]
            part = part if torch.is_tensor(part) else torch.from_numpy(np.ascontiguousarray(part))
            self.feats[r0:r0 + part.shape[0]].copy_(part.to(dtype))
        self._init_index(dev, sizes, offsets, labels)

    def _init_index(self, dev, sizes, offsets, labels):
        self.device = dev
        self.sizes = sizes
        self.offsets = offsets
        self.sizes_d = torch.from_numpy(sizes.astype(np.int32)).to(dev)
        self.offsets_d = torch.from_numpy(offsets).to(dev)
        self.labels = None if labels is None else np.asarray(labels, dtype=np.int64).reshape(-1)
        if self.labels is not None and self.labels.shape != sizes.shape:
            raise ValueError("one label per sample")
        self.labels_d = None if self.labels is None else torch.from_numpy(self.labels).to(dev)

    def __len__(self):
        return len(self.sizes)

    @classmethod
    def concat(cls, stores):
        """One store over several (e.g. IEMOCAP + CASIA + EMODB for mixed batches): frames
        concatenated in HBM (one device copy), offsets shifted, labels kept.  Sample i of
        stores[k] becomes sample starts[k] + i; returns (store, starts)."""
        if not stores:
            raise ValueError("no stores")
        dev = stores[0].device
        dtype = stores[0].feats.dtype
        if any(st.feats.dtype != dtype or st.device != dev for st in stores):
            raise ValueError("stores must share dtype and device")
        out = cls.__new__(cls)
        out.feats = torch.cat([st.feats for st in stores], 0)
        base = np.cumsum([0] + [st.feats.shape[0] for st in stores])[:-1]
        starts = np.cumsum([0] + [len(st) for st in stores])
        labeled = all(st.labels is not None for st in stores)
        out._init_index(dev, np.concatenate([st.sizes for st in stores]),
                        np.concatenate([st.offsets + b for st, b in zip(stores, base)]),
                        np.concatenate([st.labels for st in stores]) if labeled else None)
        return out, starts[:-1]

    def subset(self, indices, with_labels=True):
        """create_subset (I/dataload_noisy.py:193-205, C/dataload_casia_noisy.py:200-224): the
        samples `indices` in that order, sharing this store's rows (no copy)."""
        idx = np.asarray(indices, dtype=np.int64).reshape(-1)
        sub = FeatureStore.__new__(FeatureStore)
        sub.feats = self.feats
        labels = self.labels[idx] if (with_labels and self.labels is not None) else None
        sub._init_index(self.device, self.sizes[idx], self.offsets[idx], labels)
        return sub

    def collate(self, index, index_d=None, T=None, style="iemocap", with_labels=True, stream=None):
        """One batch, as the reference collator returns it (I/dataload_noisy.py:116-129):
        {'id': int64 [B], 'net_input': {'feats': f32 [B, T, 768] zero-padded,
        'padding_mask': bool [B, T] (True = pad)}, 'labels': int64 [B] or None}, on the device
        (style 'casia': the CASIA/EMODB noisy collators' dict, without 'id').
        `index` (host ints) gives T = max size; `index_d` (device int64) is used when given."""
        index = np.asarray(index, dtype=np.int64).reshape(-1)
        B = len(index)
        if B == 0:
            return {}
        if index.min() < 0 or index.max() >= len(self):
            raise IndexError("sample index out of range [0, %d)" % len(self))
        if T is None:
            T = int(self.sizes[index].max())
        if T <= 0:
            raise ValueError("every sample of the batch is empty")
        if index_d is None:
            index_d = torch.from_numpy(index).to(self.device, non_blocking=True)
        feats = torch.empty(B, T, 768, dtype=torch.float32, device=self.device)
        pad = torch.empty(B, T, dtype=torch.uint8, device=self.device)
        lab = None
        if with_labels and self.labels_d is not None:
            lab = torch.empty(B, dtype=torch.int64, device=self.device)
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _lib.check(_lib.lib().dad_collate(
            _lib.ptr(self.feats), STORE_DTYPES[self.feats.dtype], _lib.ptr(self.offsets_d), _lib.ptr(self.sizes_d),
            len(self), _lib.ptr(index_d), B, T, _lib.ptr(feats), _lib.ptr(pad),
            _lib.ptr(self.labels_d if lab is not None else None), _lib.ptr(lab), s.cuda_stream), "dad_collate")
        return self._pack(index_d, feats, pad, lab, style)

    def batch_index(self, index, index_d=None, T=None, style="iemocap", with_labels=True, stream=None):
        """Store-mode batch (no feature copy): the collator's dict with net_input['feats'] a
        StoreFeats over this store; padding mask and labels as collate() writes them
        (dad_collate_index)."""
        index = np.asarray(index, dtype=np.int64).reshape(-1)
        B = len(index)
        if B == 0:
            return {}
        if index.min() < 0 or index.max() >= len(self):
            raise IndexError("sample index out of range [0, %d)" % len(self))
        if T is None:
            T = int(self.sizes[index].max())
        if index_d is None:
            index_d = torch.from_numpy(index).to(self.device, non_blocking=True)
        rows = torch.empty(B, dtype=torch.int64, device=self.device)
        lens = torch.empty(B, dtype=torch.int32, device=self.device)
        pad = torch.empty(B, T, dtype=torch.uint8, device=self.device)
        lab = None
        if with_labels and self.labels_d is not None:
            lab = torch.empty(B, dtype=torch.int64, device=self.device)
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _lib.check(_lib.lib().dad_collate_index(
            _lib.ptr(self.offsets_d), _lib.ptr(self.sizes_d), len(self), _lib.ptr(index_d), B, T, _lib.ptr(rows),
            _lib.ptr(lens), _lib.ptr(pad), _lib.ptr(self.labels_d if lab is not None else None), _lib.ptr(lab),
            s.cuda_stream), "dad_collate_index")
        return self._pack(index_d, StoreFeats(self, index, index_d, rows, lens, T), pad, lab, style)

    @staticmethod
    def _pack(index_d, feats, pad, lab, style):
        net_input = {"feats": feats, "padding_mask": pad if pad.dtype == torch.bool else pad.view(torch.bool)}
        if style == "casia":           # C/dataload_casia_noisy.py:93-106: no 'id'; 'labels' only when labeled
            return {"net_input": net_input, **({"labels": lab} if lab is not None else {})}
        return {"id": index_d, "net_input": net_input, "labels": lab}


class StoreFeats:
    """net_input['feats'] of a store-mode batch: B utterances of a FeatureStore at padded
    length T, NOT copied -- DADStep hands the store and the per-utterance rows/lengths to the
    encoder, whose LDS-DMA reads the rows in place (dad_batch store mode, include/dad.h).
    .shape is the padded batch's; .materialize() returns the padded f32 tensor (dad_collate)."""

    def __init__(self, store, index, index_d, rows, lens, T):
        self.store, self.index, self.index_d, self.rows, self.lens = store, index, index_d, rows, lens
        self.shape = torch.Size((len(index), T, 768))
        self.dtype = torch.float32
        self.device = store.device

    def dim(self):
        return 3

    def materialize(self):
        return self.store.collate(self.index, index_d=self.index_d, T=self.shape[1],
                                  with_labels=False)["net_input"]["feats"]


class DeviceLoader:
    """torch DataLoader(dataset, batch_size, shuffle, collate_fn=dataset.collator) over a
    FeatureStore, collating on the device.  `style`: 'iemocap' (the I/ collators' dict, with
    'id') or 'casia' (C/ and E/ noisy collators: no 'id', 'labels' only when labeled);
    `with_labels`: False for the reference's unlabeled SSL training loaders; `fused`: yield
    store-mode batches (StoreFeats, no feature copy) that DADStep feeds to the encoder's
    row gather -- the padded feature tensor never exists."""

    def __init__(self, store, batch_size=1, shuffle=False, generator=None, drop_last=False, style="iemocap",
                 with_labels=True, fused=False):
        self.store = store
        self.fused = fused
        self.dataset = store
        self.batch_size = batch_size
        self.style = style
        self.with_labels = with_labels and store.labels is not None
        self._pinned = self._pin_ev = None      # _upload's pinned staging buffer
        self._index_loader = torch.utils.data.DataLoader(range(len(store)), batch_size=batch_size, shuffle=shuffle,
                                                         generator=generator, drop_last=drop_last,
                                                         collate_fn=_identity, num_workers=0)

    def __len__(self):
        return len(self._index_loader)

    def __iter__(self):
        return _DeviceLoaderIter(self)

    def _upload(self, host, dev):
        """int64 array -> a new device tensor, asynchronously through this loader's pinned buffer
        (allocated once: pinning per epoch called the host allocator each time; an event keeps the
        buffer from being refilled before the previous copy has read it)."""
        t = torch.from_numpy(np.ascontiguousarray(host, dtype=np.int64))
        if dev.type != "cuda":
            return t.to(dev)
        if self._pinned is None or self._pinned.numel() < t.numel():
            self._pinned = torch.empty(max(t.numel(), 1), dtype=torch.int64).pin_memory()
            self._pin_ev = None
        if self._pin_ev is not None:
            self._pin_ev.synchronize()
        buf = self._pinned[:t.numel()]
        buf.copy_(t)
        out = torch.empty(t.numel(), dtype=torch.int64, device=dev)
        out.copy_(buf, non_blocking=True)
        self._pin_ev = torch.cuda.Event()
        self._pin_ev.record(torch.cuda.current_stream(dev))
        return out


def _identity(batch):
    return batch


def _fast_batches(dl):
    """The batches one epoch of DataLoader(range(n), batch_size, shuffle, generator, drop_last)
    yields, without its per-index Python iteration (≈0.5 us per sample, ≈30 us per batch of 64):
    for the default samplers, the same draws in the same order -- RandomSampler's seed from the
    global RNG (or its generator) and one randperm -- cut into batch_size chunks as BatchSampler
    does.  None for any other sampler (the caller drains the DataLoader).  The iterator's own base
    seed was drawn when the caller created it (iter(DataLoader)), as before."""
    bs = dl.batch_sampler
    if type(bs) is not torch.utils.data.BatchSampler or dl.num_workers != 0:
        return None
    smp = bs.sampler
    n = len(dl.dataset)
    if type(smp) is torch.utils.data.SequentialSampler:
        order = np.arange(n, dtype=np.int64)
    elif (type(smp) is torch.utils.data.RandomSampler and not smp.replacement and smp.num_samples == n
          and smp._num_samples is None):
        g = smp.generator
        if g is None:
            seed = int(torch.empty((), dtype=torch.int64).random_().item())
            g = torch.Generator()
            g.manual_seed(seed)
        order = torch.randperm(n, generator=g).numpy().astype(np.int64)
        # RandomSampler's trailing `randperm(n)[: num_samples % n]` runs when the epoch is drained
        # (an empty slice, but a caller's generator advances)
        torch.randperm(n, generator=g)
    else:
        return None
    k = bs.batch_size
    stop = (n // k) * k if bs.drop_last else n
    return [order[i:i + k] for i in range(0, stop, k)]


class _DeviceLoaderIter:
    def __init__(self, loader):
        self.loader = loader
        self._it = iter(loader._index_loader)     # the reference's iter(): same global-RNG draw
        self._batches = None
        self._k = 0
        self._rows = None           # store mode: the epoch's rows / lengths / masks / labels (_epoch_index)

    def __iter__(self):
        return self

    def __next__(self):
        L = self.loader
        if self._batches is None:
            # the sampler draws its permutation at the first next(), as in the reference
            self._batches = _fast_batches(L._index_loader)
            if self._batches is None:
                self._batches = [np.asarray(b, dtype=np.int64) for b in self._it]
            flat = np.concatenate(self._batches) if self._batches else np.zeros(0, np.int64)
            dev = torch.device(L.store.device)
            sizes = np.fromiter((len(b) for b in self._batches), np.int64, len(self._batches))
            self._starts = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
            n = len(flat)
            # each batch's T = its longest sample (one reduceat over the epoch, empty batches 0)
            Tk = np.zeros(len(sizes), np.int64)
            if n:
                ne = sizes > 0
                Tk[ne] = np.maximum.reduceat(np.asarray(L.store.sizes)[flat], self._starts[:-1][ne])
            self._T = Tk.tolist()
            epoch = L.fused and dev.type == "cuda" and n > 0 and min(self._T) > 0
            if epoch:   # store mode: the epoch's per-sample pad offsets and T go up with the index
                if flat.min() < 0 or flat.max() >= len(L.store):
                    raise IndexError("sample index out of range [0, %d)" % len(L.store))
                self._pad_off = np.concatenate([[0], np.cumsum(sizes * Tk)]).astype(np.int64)
                Ts = np.repeat(Tk, sizes)            # each sample's T; its pad row follows the previous row's
                host = np.concatenate([flat, np.concatenate([[0], np.cumsum(Ts)[:-1]]), Ts])
            else:
                host = flat
            # one upload per epoch, asynchronous, from the loader's pinned buffer (a pageable copy
            # waits for every step already queued on the stream: a pipeline drain per epoch)
            up = L._upload(host, dev)
            self._index_d = up[:n]
            if epoch:
                self._epoch_index(up)
        if self._k >= len(self._batches):
            raise StopIteration
        k = self._k
        self._k += 1
        b = self._batches[k]
        s0, s1 = self._starts[k], self._starts[k + 1]
        if self._rows is not None:   # store mode: this batch's views of the epoch's index tensors
            idx_d, rows, lens, pad, lab = self._views[k]
            feats = StoreFeats(L.store, b, idx_d, rows, lens, self._T[k])
            return FeatureStore._pack(idx_d, feats, pad, lab, L.style)
        fn = L.store.batch_index if L.fused else L.store.collate
        return fn(b, index_d=self._index_d[s0:s1], T=self._T[k], style=L.style, with_labels=L.with_labels)

    def _epoch_index(self, up):
        """Store mode: what FeatureStore.batch_index writes per batch (store rows, lengths, padding
        mask at the batch's own T, labels), for every batch of the epoch at its first next(), in one
        launch (dad_collate_index_epoch) into epoch-sized buffers the batches are views of.  Per batch
        that replaces four device allocations and a library call on the host (~35 us, two loaders per
        train step, which kept the store-fed step host-bound) with a few tensor views."""
        L = self.loader
        st = L.store
        dev = torch.device(st.device)
        n = int(self._starts[-1])
        self._rows = torch.empty(n, dtype=torch.int64, device=dev)
        self._lens = torch.empty(n, dtype=torch.int32, device=dev)
        self._pad = torch.empty(int(self._pad_off[-1]), dtype=torch.bool, device=dev)
        self._lab = None
        if L.with_labels and st.labels_d is not None:
            self._lab = torch.empty(n, dtype=torch.int64, device=dev)
        _lib.check(_lib.lib().dad_collate_index_epoch(
            _lib.ptr(st.offsets_d), _lib.ptr(st.sizes_d), len(st), _lib.ptr(up[:n]), n, _lib.ptr(up[n:2 * n]),
            _lib.ptr(up[2 * n:]), _lib.ptr(self._rows), _lib.ptr(self._lens), _lib.ptr(self._pad),
            _lib.ptr(st.labels_d if self._lab is not None else None), _lib.ptr(self._lab),
            torch.cuda.current_stream(dev).cuda_stream), "dad_collate_index_epoch")
        # every batch's views, made here by one split per buffer (C++: well under a microsecond per view)
        # instead of per next() (five Python slicings and a reshape, ~30 us per batch: with two loaders per
        # train step that was half of the store-fed step's host time, which bounded it)
        sizes = [int(x) for x in np.diff(self._starts)]
        nb = len(sizes)
        sp = lambda t: t.split(sizes) if t is not None else [None] * nb
        pads = [c.view(sz, T) for c, sz, T in zip(self._pad.split([s * T for s, T in zip(sizes, self._T)]), sizes,
                                                   self._T)]
        self._views = list(zip(sp(self._index_d), sp(self._rows), sp(self._lens), pads, sp(self._lab)))


# ------------------------------------------------------------------- reference file formats

def load_emotion2vec_dataset(data_path, labels="emo", min_length=3, max_length=None, ignore_labels=False):
    """I/dataload_noisy.py:67-90: (features, sizes, offsets, label names).  Samples outside
    [min_length, max_length] are skipped but advance the running offset (kept offsets index
    the original array).  The .npy is memory-mapped (no unpickling, no full host copy)."""
    npy = np.load(data_path + ".npy", mmap_mode="r")
    sizes, offsets, names = [], [], []
    lbl_path = data_path + "." + labels
    use_labels = not ignore_labels and os.path.exists(lbl_path)
    offset = 0
    with open(data_path + ".lengths") as len_f, (open(lbl_path) if use_labels else contextlib.ExitStack()) as lbl_f:
        for line in len_f:
            n = int(line.rstrip())
            name = next(lbl_f).rstrip().split()[1] if use_labels else None
            if n >= min_length and (max_length is None or n <= max_length):
                sizes.append(n)
                offsets.append(offset)
                if name is not None:
                    names.append(name)
            offset += n
    return npy, np.asarray(sizes), np.asarray(offsets), (None if ignore_labels else names)


def iemocap_fold_split(session_ids, fold_id):
    """(train, val, test) sample indices of an IEMOCAP session fold (I/dataload_noisy.py:44-65,
    193-205)."""
    return _session_subsets(np.asarray(session_ids), fold_id)


def casia_fold_split(speakers, fold):
    """(train, val, test) indices of a CASIA speaker fold (C/dataload_casia_noisy.py:175-182),
    train in index order (the loaders shuffle)."""
    spk = np.unique(speakers)
    test_spk, val_spk = spk[fold % len(spk)], spk[(fold + 1) % len(spk)]
    tr = np.where(~np.isin(speakers, [test_spk, val_spk]))[0]
    return tr, np.where(speakers == val_spk)[0], np.where(speakers == test_spk)[0]


def emodb_fold_split(speakers, fold):
    """(train, val, test) indices of an EMODB leave-one-speaker-out fold (E/dataload_emodb_noisy.py:23-47)."""
    tr_spk, va_spk, te_spk = get_emodb_fold_speakers(fold)
    ids = np.array([str(s).split("_")[-1] for s in speakers])
    return np.where(np.isin(ids, tr_spk))[0], np.where(ids == va_spk)[0], np.where(ids == te_spk)[0]


def get_session_ids(data_path, num_samples):
    """I/dataload_noisy.py:17-42 (the session digit is character 4 of each .emo line's name)."""
    path = data_path + ".emo"
    if not os.path.exists(path):
        return [None] * num_samples
    with open(path, encoding="utf-8") as f:
        return [int(ln.strip().split("\t")[0].strip()[4]) for ln in f if ln.strip()]


def get_fold_sessions(fold_id):
    """I/dataload_noisy.py:44-65: (train sessions, val session, test session)."""
    folds = {1: ([1, 2, 3], 4, 5), 2: ([2, 3, 4], 5, 1), 3: ([3, 4, 5], 1, 2), 4: ([4, 5, 1], 2, 3),
             5: ([5, 1, 2], 3, 4)}
    if fold_id not in folds:
        raise ValueError(f"fold_id must be between 1 and 5, got {fold_id}")
    return folds[fold_id]


def load_ssl_features(feature_path, label_dict=IEMOCAP_LABEL_DICT, device=None, dtype=None):
    """I/dataload_noisy.py:131-153: <feature_path>/train.*, all samples (min_length 1), as a
    FeatureStore plus the per-sample session ids."""
    data_path = os.path.join(feature_path, "train")
    npy, sizes, offsets, names = load_emotion2vec_dataset(data_path, labels="emo", min_length=1)
    labels = [label_dict[x] for x in names] if names else None
    num = len(labels) if labels else len(sizes)
    store = FeatureStore(npy, sizes, offsets, labels, device=device, dtype=dtype)
    return store, np.array(get_session_ids(data_path, num))


def _session_subsets(session_ids, fold_id):
    tr_s, va_s, te_s = get_fold_sessions(fold_id)
    return (np.where(np.isin(session_ids, tr_s))[0], np.where(session_ids == va_s)[0],
            np.where(session_ids == te_s)[0])


def get_cv_dataloaders(data_path, batch_size=64, fold_id=1, device=None, dtype=None):
    """Clean loaders, I/dataload_clean.py:222-293: (train [shuffled], val, test, class_names,
    num_classes), all labeled, batches with 'id'."""
    store, sess = load_ssl_features(data_path, device=device, dtype=dtype)
    tr, va, te = _session_subsets(sess, fold_id)
    out = (DeviceLoader(store.subset(tr), batch_size, shuffle=True),
           DeviceLoader(store.subset(va), batch_size, shuffle=False),
           DeviceLoader(store.subset(te), batch_size, shuffle=False))
    return out + (list(IEMOCAP_LABEL_DICT), len(IEMOCAP_LABEL_DICT))


def get_cv_dataloaders_noisy(data_path, batch_size=64, fold_id=1, device=None, dtype=None):
    """Noisy loaders, I/dataload_noisy.py:159-231: (student, teacher [both shuffled, unlabeled:
    labels None], val, test [labeled])."""
    store, sess = load_ssl_features(data_path, device=device, dtype=dtype)
    tr, va, te = _session_subsets(sess, fold_id)
    train = store.subset(tr, with_labels=False)
    return (DeviceLoader(train, batch_size, shuffle=True), DeviceLoader(train, batch_size, shuffle=True),
            DeviceLoader(store.subset(va), batch_size, shuffle=False),
            DeviceLoader(store.subset(te), batch_size, shuffle=False))


def load_casia_noisy_data(feature_path, label_dict=CASIA_LABEL_DICT, device=None, dtype=None):
    """C/dataload_casia_noisy.py:109-158: <prefix>.{npy,lengths,lbl,spk}; returns the store and
    the per-sample speaker names."""
    npy = np.load(feature_path + ".npy", mmap_mode="r")
    with open(feature_path + ".lengths") as f:
        sizes = np.array([int(x.strip()) for x in f], dtype=np.int64)
    with open(feature_path + ".lbl", encoding="utf-8") as f:
        labels = [label_dict[x.strip()] for x in f]
    with open(feature_path + ".spk", encoding="utf-8") as f:
        speakers = np.array([x.strip() for x in f])
    offsets = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    return FeatureStore(npy, sizes, offsets, labels, device=device, dtype=dtype), speakers


def create_casia_noisy_speaker_isolated_loaders(store, speakers, fold, batch_size):
    """C/dataload_casia_noisy.py:160-292: 4 speakers; test = sorted speaker[fold], val = the
    next, train = the other two, the train indices shuffled with the global NumPy RNG (as the
    reference does) before the loaders shuffle again.  Batches have no 'id'; the two train
    loaders are unlabeled."""
    spk = np.unique(speakers)
    if len(spk) != 4:
        raise ValueError(f"expected 4 CASIA speakers, found {len(spk)}")
    test_spk, val_spk = spk[fold], spk[(fold + 1) % 4]
    tr = np.where(np.isin(speakers, [s for s in spk if s not in [test_spk, val_spk]]))[0]
    np.random.shuffle(tr)
    va, te = np.where(speakers == val_spk)[0], np.where(speakers == test_spk)[0]
    mk = lambda idx, lab, sh: DeviceLoader(store.subset(idx, with_labels=lab), batch_size, shuffle=sh, style="casia")
    return mk(tr, False, True), mk(tr, False, True), mk(va, True, False), mk(te, True, False)


EMODB_SPEAKERS = ['03', '08', '09', '10', '11', '12', '13', '14', '15', '16']   # E/dataload_emodb_noisy.py:21


def get_emodb_fold_speakers(fold_id):
    """E/dataload_emodb_noisy.py:23-47: (8 train speakers, val = next speaker, test = speaker[fold])."""
    if fold_id < 0 or fold_id >= 10:
        raise ValueError(f"fold_id must be between 0 and 9, got {fold_id}")
    test_spk, val_spk = EMODB_SPEAKERS[fold_id], EMODB_SPEAKERS[(fold_id + 1) % 10]
    return [s for s in EMODB_SPEAKERS if s not in [test_spk, val_spk]], val_spk, test_spk


def load_emodb_noisy_data(feature_path, label_dict=CASIA_LABEL_DICT, device=None, dtype=None):
    """E/dataload_emodb_noisy.py:140-189: same files as CASIA (.npy/.lengths/.lbl/.spk)."""
    return load_casia_noisy_data(feature_path, label_dict, device=device, dtype=dtype)


def create_emodb_noisy_speaker_isolated_loaders(store, speakers, fold, batch_size):
    """E/dataload_emodb_noisy.py:191-342: speakers matched on the part after the last '_'
    ('emodb_spk_03' -> '03'); 10 folds; the train indices shuffled with the global NumPy RNG;
    batches without 'id', the two train loaders unlabeled."""
    if fold < 0 or fold >= 10:
        raise ValueError(f"fold must be in 0-9, got {fold}")
    tr_spk, va_spk, te_spk = get_emodb_fold_speakers(fold)
    ids = np.array([s.split("_")[-1] for s in speakers])
    tr = np.where(np.isin(ids, tr_spk))[0]
    va, te = np.where(ids == va_spk)[0], np.where(ids == te_spk)[0]
    np.random.shuffle(tr)
    for name, idx in (("train", tr), ("val", va), ("test", te)):
        if len(idx) == 0:
            raise ValueError("no samples for the %s subset" % name)
    mk = lambda idx, lab, sh: DeviceLoader(store.subset(idx, with_labels=lab), batch_size, shuffle=sh, style="casia")
    return mk(tr, False, True), mk(tr, False, True), mk(va, True, False), mk(te, True, False)
