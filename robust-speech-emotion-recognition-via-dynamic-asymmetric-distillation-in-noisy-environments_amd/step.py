"""The fused DAD train step: one C-ABI call sequence per step, all decisions on device.

`DADStep.step(clean_batch, noisy_batch, epoch)` replaces the body of the reference's
`train_epoch` loop (I/train.py:484-492):

    optimizer.zero_grad(); losses = train_step(clean, noisy, epoch)      # I/train.py:397-471
    losses['total_loss'].backward(); clip_grad_norm_(...); optimizer.step()
    if not warm-up: model.update_teacher_ema()

with the same batch dicts (`{'net_input': {'feats', 'padding_mask'}, 'labels'}`,
I/dataload_noisy.py:124-129) and the same returned loss dict keys.  The step keeps the
Adam moments, the DACP state (`DACPManager`: ema_thresholds, class_quality_scores, epoch
score statistics) and every scratch buffer on the device; nothing is synchronised with the
host, so losses come back as 0-d device tensors.
"""
import ctypes

import torch

from . import _lib
from .config import ConfigCache, ConfigView
from .data import StoreFeats

PRECISIONS = {"fp32": _lib.PREC_FP32, "bf16": _lib.PREC_BF16, "fp16": _lib.PREC_FP16}


def _dev_batch(batch, device, labels=True):
    """(x, pad, y, rows, lens): a padded batch, or a store-mode batch (data.StoreFeats: x is the
    feature store and rows/lens locate each utterance in it, dad_batch.rowc..lenn)."""
    ni = batch["net_input"]
    feats = ni["feats"]
    rows = lens = None
    if isinstance(feats, StoreFeats):
        sf = feats.store.feats
        if sf.dtype == torch.float32 and sf.device == device:
            x, rows, lens = sf, feats.rows, feats.lens
        else:                      # the encoders read f32 rows: other stores are widened by dad_collate
            x = feats.materialize().to(device)
        pm = ni["padding_mask"]
        # (the loaders' own tensors need no conversion: skip the no-op .to()/.contiguous() dispatches)
        if not (pm.dtype == torch.bool and pm.device == device and pm.is_contiguous()):
            pm = pm.to(device=device, dtype=torch.bool).contiguous()
        pad = pm.view(torch.uint8)
        y = None
        if labels:
            y = batch["labels"]
            if not (y.dtype == torch.int64 and y.device == device and y.is_contiguous()):
                y = y.to(device=device, dtype=torch.int64).contiguous()
        return x, pad, y, rows, lens
    x = feats.to(device=device, dtype=torch.float32, non_blocking=True).contiguous()
    pm = ni.get("padding_mask")
    if pm is None:
        pad = torch.zeros(x.shape[0], x.shape[1], dtype=torch.uint8, device=device)
    else:
        pad = pm.to(device=device, dtype=torch.bool, non_blocking=True).contiguous().view(torch.uint8)
    y = None
    if labels:
        y = batch["labels"].to(device=device, dtype=torch.int64, non_blocking=True).contiguous()
    if x.dim() != 3 or x.shape[2] != 768:
        raise ValueError("feats must be [B, T, 768], got %s" % (tuple(x.shape),))
    return x, pad, y, None, None


def _resident(batch, device, labels=True):
    """True when _dev_batch hands out the batch's own device tensors (no copy), i.e. the pointers a
    step would prepare ahead are the ones the next step will see: f32 features (or an f32 store) on
    `device`, a bool padding mask and int64 labels there, all contiguous."""
    ni = batch["net_input"]
    feats, pm = ni["feats"], ni.get("padding_mask")
    if isinstance(feats, StoreFeats):
        ok = feats.store.feats.dtype == torch.float32 and feats.store.feats.device == device
    else:
        ok = (torch.is_tensor(feats) and feats.device == device and feats.dtype == torch.float32
              and feats.is_contiguous())
    ok = ok and torch.is_tensor(pm) and pm.device == device and pm.dtype == torch.bool and pm.is_contiguous()
    if labels:
        y = batch["labels"]
        ok = ok and torch.is_tensor(y) and y.device == device and y.dtype == torch.int64 and y.is_contiguous()
    return bool(ok)


_DRAW_DTYPES = {"nw": torch.float32, "ns": torch.float32, "u": torch.float32, "start": torch.int64,
                "keep1": torch.bool, "keep2": torch.bool}


def _draws_resident(draws, device):
    """Explicit draws that _batch_structs uses in place (same dtype, on `device`, contiguous)."""
    if draws is None:
        return False
    for k, dt in _DRAW_DTYPES.items():
        v = draws.get(k)
        if v is not None and not (torch.is_tensor(v) and v.device == device and v.dtype == dt and v.is_contiguous()):
            return False
    return True


class _StepLossFn(torch.autograd.Function):
    """total_loss whose backward hands the step's analytic gradient to the student params.

    forward(loss, flat_grad, W1, b1, W2, b2) -> loss; d(loss)/d(param) = slices of flat_grad
    (computed by the fused kernels against the parameters the forward saw)."""

    @staticmethod
    def forward(ctx, loss, flat_grad, *params):
        ctx.save_for_backward(flat_grad)
        ctx.shapes = [p.shape for p in params]
        return loss.detach().clone()

    @staticmethod
    def backward(ctx, g):
        (flat,) = ctx.saved_tensors
        out, off = [], 0
        for shp in ctx.shapes:
            n = 1
            for d in shp:
                n *= d
            out.append((flat[off:off + n] * g).view(shp))
            off += n
        return (None, None, *out)


class DADStep:
    """Owns the device state of the DAD step around an `SSRLModel`.

    Args:
        model: `SSRLModel` (already on the target cuda device).
        cfg: reference-style config module / dict / object (read at every step), or None.
        flavor: 'iemocap' | 'casia' | 'emodb' (which ablation switches are honoured).
        precision: 'fp32' (exact-f32 MFMA, the reference's arithmetic), 'fp16' (fp16 MFMA operands,
            fp32 accumulate: the throughput mode that keeps losses and logits within 1e-4) or
            'bf16' (bf16 operands, fp32 accumulate).
        rng: 'counter' (in-kernel counter-based RNG) or 'explicit' (draws passed to step()).
        seed: counter-RNG seed.
        comm: optional `dist.DPComm` for data-parallel gradient averaging.
        prep_under_exchange: 16-bit steps that name their next batch: which of its rows are prepared
            on a second stream from the end of the backward on, i.e. under the gradient all-reduce
            (dad_step_backward_ahead_split), instead of inside this step's launches: 0 / False (none,
            the default), True (= the clean rows: the weight gradient then runs as the plain GEMM), or a
            mask of _lib.PREP_CLEAN / PREP_NOISY.  Results are bit-identical either way.  Measured on
            one MI355X with a spin standing in for the exchange window (bench.py --exchange-us, DESIGN
            section 5): the side-stream layouts cost 21-40 us per step against the in-launch layout at
            windows of 0-20 us (the two cross-stream hops and the standalone preparation are exposed),
            so nothing is moved by default at any N; the option is for longer exchange windows.
    """

    def __init__(self, model, cfg=None, flavor=None, precision="fp32", rng="counter", seed=0, comm=None,
                 anchors=None, splits=0, prep_under_exchange=None):
        self.model = model
        self.view = cfg if isinstance(cfg, ConfigView) else ConfigView(cfg, flavor=flavor)
        self.device = model.student_flat.device
        if self.device.type != "cuda":
            raise RuntimeError("DADStep needs the model on an MI355X ('cuda') device")
        self.precision = PRECISIONS[precision]
        self.rng_mode = _lib.RNG_COUNTER if rng == "counter" else _lib.RNG_EXPLICIT
        self.seed = int(seed)
        self.comm = comm
        self.splits = int(splits)
        dev = self.device
        P = _lib.DAD_NPARAM
        self.exp_avg = torch.zeros(P, device=dev)
        self.exp_avg_sq = torch.zeros(P, device=dev)
        self.grad = torch.zeros(_lib.DAD_GRAD_FLOATS, device=dev)
        self.w1bf_student = torch.empty(256 * 768, dtype=torch.bfloat16, device=dev)
        self.w1bf_teacher = torch.empty(256 * 768, dtype=torch.bfloat16, device=dev)
        # DACPManager state (I/utils.py:384-398): tau=0.5, Q=0.5, epoch sums, anchors
        self.dacp = torch.zeros(_lib.DAD_DACP_FLOATS, device=dev)
        self.dacp[0:4] = 0.5
        self.dacp[4:8] = 0.5
        if anchors is not None:
            self.set_anchors(anchors)
        self.adam_step = 0
        self.global_step = 0
        self._ws = None
        self._ws_need = {}       # workspace bytes per layout key (_workspace)
        self._cfg_cache = ConfigCache()   # dad_config_for's step-independent part (config.py)
        self._bufs = {}
        self._prepped_key = None       # identity of the batch the last step's tail launch prepared
        self.last_prepped = False
        self._next_keep = None
        self._shadow_dirty = False
        self.prep_under_exchange = 0 if prep_under_exchange is None else prep_under_exchange
        self._side = None            # the side stream of the preparation under the exchange
        self._prep_event = None      # recorded after it: the next step's encoder waits for it
        self.refresh_shadow()

    # ----------------------------------------------------------------------------- state
    @property
    def ema_thresholds(self):
        return self.dacp[0:4]

    @property
    def class_quality_scores(self):
        return self.dacp[4:8]

    @property
    def calibrated_anchors(self):
        return self.dacp[16:20]

    def set_anchors(self, anchors):
        """`calibrated_anchors` input of DACPManager.calculate_mask (I/train.py:317-357)."""
        a = torch.as_tensor(anchors, dtype=torch.float32).to(self.device)
        self.dacp[16:20].copy_(a)

    def _param_key(self):
        """Identity + write count of the model's flat parameter vectors.  In-place writes to
        the parameters themselves (load_state_dict, optimizer steps, `p.copy_`) bump the shared
        version counter; kernel writes made outside this step (SSRLModel.update_teacher_ema)
        bump `model.param_writes`; `.to()` rebinds the storage.

        NOT detected: writes through `p.data` (`p.data.copy_(...)`, the style of the
        reference's model.py:204-223).  `.data` is a detached alias with a version counter of
        its own, so such a write leaves this key unchanged and the next FP16/BF16 step would run
        on the old 16-bit W1 shadows.  Call `refresh_shadow()` after writing through `.data`
        (tests/test_gpu_shadow.py).  A per-step content check would cost a read of both W1
        copies (1.5 MB) on every step."""
        m = self.model
        s, t = m.student_flat, m.teacher_flat
        return (s.data_ptr(), t.data_ptr(), s._version, t._version, getattr(m, "param_writes", 0))

    def refresh_shadow(self):
        """Re-derive the 16-bit W1 shadows after the caller changed the model's parameters
        (step() also does this by itself whenever `_param_key` changed; required after writes
        through `.data`, which `_param_key` cannot see)."""
        st = self._state_struct(0)
        _lib.check(_lib.lib().dad_refresh_shadow(st, self.precision, self._stream()), "dad_refresh_shadow")
        self._shadow_dirty = False
        self._shadow_key = self._param_key()

    def state_dict(self):
        return {"exp_avg": self.exp_avg.clone(), "exp_avg_sq": self.exp_avg_sq.clone(),
                "adam_step": self.adam_step, "global_step": self.global_step, "dacp": self.dacp.clone()}

    def load_state_dict(self, sd):
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.adam_step = int(sd["adam_step"])
        self.global_step = int(sd.get("global_step", 0))
        self.dacp.copy_(sd["dacp"])

    # ---------------------------------------------------------------------------- buffers
    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def _buffers_for(self, Bc, Bn):
        key = (Bc, Bn)
        b = self._bufs.get(key)
        if b is None:
            dev = self.device
            nb = Bc + 2 * Bn
            b = {"tail": torch.zeros(_lib.tail_floats(max(Bn, 1)), device=dev),
                 "emb": torch.zeros(max(nb, 1), 256, device=dev),
                 "logits": torch.zeros(max(nb, 1), 4, device=dev)}
            self._bufs[key] = b
        return b

    def _state_struct(self, Bn, Bc=None):
        m = self.model
        s = _lib.DadState()
        s.student = m.student_flat.data_ptr()
        s.teacher = m.teacher_flat.data_ptr()
        s.exp_avg = self.exp_avg.data_ptr()
        s.exp_avg_sq = self.exp_avg_sq.data_ptr()
        s.grad = self.grad.data_ptr()
        s.w1bf_student = self.w1bf_student.data_ptr()
        s.w1bf_teacher = self.w1bf_teacher.data_ptr()
        s.dacp = self.dacp.data_ptr()
        if Bc is not None:
            b = self._buffers_for(Bc, Bn)
            s.tail, s.emb, s.logits = b["tail"].data_ptr(), b["emb"].data_ptr(), b["logits"].data_ptr()
            self._last = b
            self._last_shape = (Bc, Bn)
        return s

    def _workspace(self, cfg):
        # dad_workspace_bytes depends on the geometry, the split count, the precision and the
        # warm-up flag only (dad_abi.hip: dad_ws_layout(geom_of, max_splits_of, precision))
        key = (cfg.B, cfg.T, cfg.Bn, cfg.Tn, cfg.splits, cfg.precision, cfg.warmup)
        need = self._ws_need.get(key)
        if need is None:
            nbytes = ctypes.c_size_t(0)
            _lib.check(_lib.lib().dad_workspace_bytes(cfg, ctypes.byref(nbytes)), "dad_workspace_bytes")
            need = self._ws_need[key] = int(nbytes.value)
        if self._ws is None or self._ws.numel() < need:
            # zero-filled once (finite bytes everywhere; the step needs no initialisation)
            self._ws = torch.zeros(need, dtype=torch.uint8, device=self.device)
        return self._ws

    # ------------------------------------------------------------------------------- step
    def make_config(self, Bc, Tc, Bn, Tn, epoch, lr=None, adam_step=None, counter=None):
        return self._cfg_cache.config(self.view, Bc, Tc, Bn, Tn, epoch,
                                      adam_step if adam_step is not None else self.adam_step + 1, lr=lr,
                                      precision=self.precision, rng_mode=self.rng_mode, seed=self.seed,
                                      counter=self.global_step if counter is None else counter,
                                      dp_world=self.comm.world if self.comm is not None else 1,
                                      splits=self.splits)

    _PREP_CFG = ("B", "T", "Bn", "Tn", "precision", "rng_mode", "seed", "counter", "warmup", "mask_len",
                 "start_hi", "weak_std", "strong_std", "feat_p")
    _PREP_BT = ("xc", "mc", "xn", "mn", "nw", "ns", "u", "start", "rowc", "lenc", "rown", "lenn")

    @classmethod
    def _prep_key(cls, cfg, bt):
        """Everything the 16-bit row preparation of a step reads (dad_prep.h): the config scalars
        and the batch's device pointers."""
        return tuple(getattr(cfg, f) for f in cls._PREP_CFG) + tuple(getattr(bt, f) for f in cls._PREP_BT)

    def _prepare(self, clean_batch, noisy_batch, epoch, lr, draws):
        """Device batch + POD structs for one step (shared by step() and train_step())."""
        cfg, bt, keep = self._batch_structs(clean_batch, noisy_batch, epoch, lr, draws)
        st = self._state_struct(cfg.Bn, cfg.B)
        self._loss_vec = torch.empty(4, device=self.device)     # written by the optimizer/commit kernel
        st.losses = self._loss_vec.data_ptr()
        self._keepalive = keep
        return cfg, bt, st

    def _batch_structs(self, clean_batch, noisy_batch, epoch, lr, draws, like=None, counter=None):
        """(dad_config, dad_batch, keepalive) of one step's batch.  like: the current step's config;
        then this is the NEXT step's batch: its config is a copy with the next counter (`counter`,
        default like's + 1; only what the row preparation reads must be right, and the preparation
        ahead needs the same geometry), or None when its geometry differs (no preparation ahead)."""
        dev = self.device
        xc, mc, yc, rc, lc = _dev_batch(clean_batch, dev)
        warm = epoch < self.view.WARMUP_EPOCHS
        rn = ln = None
        if noisy_batch is not None:
            xn, mn, _, rn, ln = _dev_batch(noisy_batch, dev, labels=False)
            Bn, Tn = mn.shape[0], mn.shape[1]
        elif warm:
            xn = mn = None
            Bn, Tn = 0, 0
        else:
            raise ValueError("post-warm-up steps need a noisy batch")
        Bc, Tc = mc.shape[0], mc.shape[1]
        if like is None:
            cfg = self.make_config(Bc, Tc, Bn, Tn, epoch, lr=lr)
        elif (like.B, like.T, like.Bn, like.Tn) == (Bc, Tc, Bn, Tn):
            cfg = _lib.DadConfig.from_buffer_copy(like)
            cfg.counter = like.counter + 1 if counter is None else counter
            cfg.prepped = 0
        else:
            return None, None, None
        bt = _lib.DadBatch()
        bt.xc, bt.mc, bt.yc = xc.data_ptr(), mc.data_ptr(), yc.data_ptr()
        if rc is not None:
            bt.rowc, bt.lenc = rc.data_ptr(), lc.data_ptr()
        if xn is not None:
            bt.xn, bt.mn = xn.data_ptr(), mn.data_ptr()
            if rn is not None:
                bt.rown, bt.lenn = rn.data_ptr(), ln.data_ptr()
        keep = []
        if self.rng_mode == _lib.RNG_EXPLICIT:
            if draws is None:
                raise ValueError("rng='explicit' needs the step's draws")
            dd = {}
            for k in ("nw", "ns", "u"):
                if draws.get(k) is not None:
                    dd[k] = torch.as_tensor(draws[k]).to(dev, torch.float32).contiguous()
            if draws.get("start") is not None:
                dd["start"] = torch.as_tensor(draws["start"]).to(dev, torch.int64).contiguous()
            for k in ("keep1", "keep2"):
                if draws.get(k) is not None:
                    dd[k] = torch.as_tensor(draws[k]).to(dev, torch.bool).contiguous().view(torch.uint8)
            for k, v in dd.items():
                setattr(bt, k, v.data_ptr())
            keep.append(dd)
        return cfg, bt, (xc, mc, yc, xn, mn, keep, rc, lc, rn, ln)

    def _ahead_ok(self, next_batch):
        """Prepare the next batch ahead only when the pointers this step would prepare from are the
        ones the next step will use: device-resident tensors (a host batch would be copied here and
        copied again by the next step, whose rows would then not match; it prepares itself)."""
        clean, noisy = next_batch[0], next_batch[1]
        if noisy is None or not (_resident(clean, self.device) and _resident(noisy, self.device, labels=False)):
            return False
        if self.rng_mode == _lib.RNG_EXPLICIT:
            return _draws_resident(next_batch[2] if len(next_batch) > 2 else None, self.device)
        return True

    def step(self, clean_batch, noisy_batch, epoch, lr=None, draws=None, after_encode=None, next_batch=None,
             next_counter=None, after_backward=None):
        """One full training step; returns the reference's loss dict as 0-d device tensors.

        after_encode: optional callable run on the host between the encoder launch and the rest
        of the step (e.g. to split a graph capture there and time the encoder with stream events).
        next_batch: optional (clean_batch, noisy_batch[, draws]) of the NEXT step (same epoch and
        lr).  FP16/BF16: its augmentation and 16-bit conversion then run inside this step's tail
        launch, on the CUs the tail leaves idle (dad_step_backward_ahead), and the next step()
        with that batch skips them.  Results are bit-identical with or without it.  Only
        device-resident batches are prepared ahead (_ahead_ok: f32 features, bool masks, int64
        labels and, with explicit draws, the draws in DADStep's dtypes, all on the step's device);
        a host batch is ignored here and copied once, by the step that runs it.  The named
        batch's device tensors must keep their contents until that step.
        after_backward: optional callable run on the host after the backward and the gradient
            exchange are enqueued, before the update (bench.py enqueues a timed spin there to stand in
            for the all-reduce window of a DP step on one GPU).
        next_counter: the next step's RNG step counter (default this step's + 1).  Graph replays
        that cycle a fixed set of captured steps pass the first captured step's counter from the
        last one (bench.capture_steps), so the cycle stays consistent.
        """
        if self._shadow_dirty or self._param_key() != self._shadow_key:
            self.refresh_shadow()
        cfg, bt, st = self._prepare(clean_batch, noisy_batch, epoch, lr, draws)
        pk, self._prepped_key = self._prepped_key, None
        cfg.prepped = 1 if (pk is not None and pk == self._prep_key(cfg, bt)) else 0
        self.last_prepped = bool(cfg.prepped)   # diagnostics: this step's rows came from the last tail launch
        self._join_side()                   # the rows prepared on the side stream under the last exchange
        ws = self._workspace(cfg)
        stream = self._stream()
        L = _lib.lib()
        _lib.check(L.dad_step_encode(cfg, bt, st, _lib.ptr(ws), stream), "dad_step_encode")
        self._next_keep = None           # (the rows it prepared were read on this stream before)
        if after_encode is not None:
            after_encode()
            stream = self._stream()
        if next_batch is not None and self.precision != _lib.PREC_FP32 and self._ahead_ok(next_batch):
            nd = next_batch[2] if len(next_batch) > 2 else None
            ncfg, nbt, nkeep = self._batch_structs(next_batch[0], next_batch[1], epoch, lr, nd, like=cfg,
                                                   counter=next_counter)
        else:
            ncfg = None
        pending = ctypes.c_int(0)
        if ncfg is not None:
            done = ctypes.c_int(0)
            defer = self._defer_parts()
            if defer:
                _lib.check(L.dad_step_backward_ahead_split(cfg, bt, st, _lib.ptr(ws), stream, ncfg, nbt, defer,
                                                           ctypes.byref(done), ctypes.byref(pending)),
                           "dad_step_backward_ahead_split")
            else:
                _lib.check(L.dad_step_backward_ahead(cfg, bt, st, _lib.ptr(ws), stream, ncfg, nbt, ctypes.byref(done)),
                           "dad_step_backward_ahead")
            if done.value:
                self._prepped_key = self._prep_key(ncfg, nbt)
                self._next_keep = nkeep          # the preparation reads these until it has run
        else:
            _lib.check(L.dad_step_backward(cfg, bt, st, _lib.ptr(ws), stream), "dad_step_backward")
        if pending.value:
            # the next batch's remaining rows on the side stream, from the end of the backward on:
            # under the all-reduce (and the optimizer), on CUs the exchange leaves idle
            main = torch.cuda.current_stream(self.device)
            if self._side is None:
                self._side = torch.cuda.Stream(self.device)
            ev = torch.cuda.Event()
            ev.record(main)
            self._side.wait_event(ev)
            _lib.check(L.dad_step_prepare_rows(ncfg, nbt, _lib.ptr(ws), self._side.cuda_stream, pending.value),
                       "dad_step_prepare_rows")
            self._prep_event = torch.cuda.Event()
            self._prep_event.record(self._side)
        if self.comm is not None and self.comm.world > 1:
            self.comm.allreduce_grad(st, stream, grad=self.grad)
        if after_backward is not None:
            after_backward()                # (bench.py: a stand-in for the exchange window at N = 1)
        if torch.cuda.is_current_stream_capturing():
            self._join_side()               # a captured graph must join its side stream itself
        _lib.check(L.dad_step_apply(cfg, st, _lib.ptr(ws), stream), "dad_step_apply")
        self.adam_step += 1
        self.global_step += 1
        return self.losses()

    def _defer_parts(self):
        """prep_under_exchange as a DAD_PREP_* mask (True: the clean rows)."""
        v = self.prep_under_exchange
        if v is True:
            return _lib.PREP_CLEAN
        return int(v or 0)

    def _join_side(self):
        """The current stream waits for the preparation issued on the side stream (if any): before
        anything reads or reallocates the workspace."""
        if self._prep_event is not None:
            torch.cuda.current_stream(self.device).wait_event(self._prep_event)
            self._prep_event = None

    def train_step(self, clean_batch, noisy_batch, epoch, draws=None):
        """Trainer.train_step (I/train.py:397-471) with an autograd-compatible total_loss.

        For callers that keep the reference loop body (I/train.py:484-492):
        `losses['total_loss'].backward()` deposits the kernels' analytic gradient into the
        student parameters' .grad, then the caller's clip_grad_norm_, optimizer.step() and
        model.update_teacher_ema() run as in the reference.  The DACP state update happens
        here, as in calculate_mask.  The other loss terms are returned detached.
        """
        if self.comm is not None and self.comm.world > 1:
            raise RuntimeError("train_step is the single-process shim; use step() with a DPComm")
        self.refresh_shadow()        # the caller's optimizer/EMA changed the fp32 params
        self._join_side()
        self._prepped_key = None     # (this step prepares its own rows into the workspace)
        cfg, bt, st = self._prepare(clean_batch, noisy_batch, epoch, None, draws)
        ws = self._workspace(cfg)
        stream = self._stream()
        L = _lib.lib()
        _lib.check(L.dad_step_compute(cfg, bt, st, _lib.ptr(ws), stream), "dad_step_compute")
        _lib.check(L.dad_step_commit(cfg, st, _lib.ptr(ws), stream), "dad_step_commit")
        self.global_step += 1
        self._shadow_dirty = True
        out = self.losses()
        m = self.model
        params = m._plist(m.student_encoder, m.student_classifier)
        out["total_loss"] = _StepLossFn.apply(out["total_loss"], self.grad[:_lib.DAD_NPARAM].clone(), *params)
        return out

    def losses(self):
        """Loss dict of the last step (keys of I/train.py:468-470 + scl_loss for CASIA/EMODB)."""
        g = self._loss_vec       # fresh per step: no copy kernels, no host sync
        out = {"total_loss": g[0], "supervised_ce_loss": g[1], "consistency_loss": g[2], "ecda_loss": g[3]}
        if self.view.flavor in ("casia", "emodb"):
            out["scl_loss"] = torch.zeros((), device=self.device)   # always 0 (C/train_CASIA.py:442)
        return out

    def range_flag(self, clear=False):
        """Device int32 scalar: the OR of the sticky range words (dad.h DAD_T_RANGE) of every batch
        shape this step has run (each (Bc, Bn) shape has its own tail buffer, so a ragged last batch
        does not hide a flag raised by the full-size batches).  Bits (`decode_range_flag`):
        RANGE_NONFINITE (1): a pooled embedding or logit was not finite (FP16: an encoder operand
        beyond +-65504; any mode: non-finite features); RANGE_POOL_TIMEOUT (2): the tail launch's
        fused pooling hand-off timed out and that step's update was skipped.  (Any step whose total
        loss is not finite leaves the parameters and state untouched.)  FP16/BF16: the encoder's
        ReLU works on the float bits (max(bits, 0)), so a NaN pre-activation with the sign bit set
        is dropped, not propagated as torch's ReLU would: NaN features can go unflagged there,
        while +-inf (an operand beyond the 16-bit range) is flagged.  `clear=True` resets every word after
        reading."""
        words = [b["tail"][_lib.T_RANGE:_lib.T_RANGE + 1].view(torch.int32) for b in self._bufs.values()]
        if not words:
            return torch.zeros((), dtype=torch.int32, device=self.device)
        v = words[0].clone()
        for w in words[1:]:
            v = torch.bitwise_or(v, w)
        if clear:
            for w in words:
                w.zero_()
        return v[0]

    @staticmethod
    def decode_range_flag(v):
        """Names of the bits set in a range_flag() value."""
        v = int(v)
        return [n for n, b in (("nonfinite", _lib.RANGE_NONFINITE), ("pool_timeout", _lib.RANGE_POOL_TIMEOUT))
                if v & b]

    def outputs(self, Bc=None, Bn=None):
        """Per-step intermediates (device tensors) of the last step, for inspection/tests."""
        b = self._last
        t = b["tail"]
        nb = (b["emb"].shape[0])
        if Bc is None:
            raise ValueError("pass Bc, Bn")
        H = _lib.DAD_TAIL_HDR
        return {
            "e_clean": b["emb"][:Bc], "e_teacher": b["emb"][Bc:Bc + Bn], "e_strong": b["emb"][Bc + Bn:Bc + 2 * Bn],
            "z_clean": b["logits"][:Bc], "z_teacher": b["logits"][Bc:Bc + Bn],
            "z_strong": b["logits"][Bc + Bn:Bc + 2 * Bn],
            "score": t[H:H + Bn], "pred": t[H + Bn:H + 2 * Bn], "mask": t[H + 2 * Bn:H + 3 * Bn],
            "q": t[H + 3 * Bn:H + 7 * Bn].view(Bn, 4) if Bn else t[H:H],
            "w": t[_lib.T_W:_lib.T_W + 4], "tau_before": t[_lib.T_TAU_BEFORE:_lib.T_TAU_BEFORE + 4],
            "tau_after": t[_lib.T_TAU_AFTER:_lib.T_TAU_AFTER + 4],
            "ecda_terms": t[_lib.T_ECDA_TERM:_lib.T_ECDA_TERM + 4],
            "clip_norm": t[_lib.T_CLIPNORM], "clip_coef": t[_lib.T_CLIPCOEF], "msum": t[_lib.T_MSUM],
            "ecda_on": t[_lib.T_ECDA_ON],
            "grad": self.grad[:_lib.DAD_NPARAM], "nb": nb,
        }

    _DRAWS = {"weak": _lib.DRAW_WEAK, "strong": _lib.DRAW_STRONG, "feat_keep": _lib.DRAW_FEAT_KEEP,
              "tstart": _lib.DRAW_TSTART, "keep1": _lib.DRAW_KEEP1, "keep2": _lib.DRAW_KEEP2}

    def counter_draws(self, which, Bc, Tc, Bn, Tn, epoch=60, counter=None, first=0, n=None):
        """The counter-RNG draws a step with this geometry makes in-kernel (dad_rng_draws):
        'weak' / 'strong' noise (std * N per element of [Bn, Tn, 768]), 'feat_keep' [768],
        'tstart' [Bn], 'keep1' [Bc*256] / 'keep2' [Bn*256] classifier dropout factors.
        `counter` defaults to the next step's (self.global_step).  Diagnostics only."""
        cfg = self.make_config(Bc, Tc, Bn, Tn, epoch)
        if counter is not None:
            cfg.counter = int(counter) & (2 ** 64 - 1)
        size = {"weak": Bn * Tn * 768, "strong": Bn * Tn * 768, "feat_keep": 768, "tstart": Bn,
                "keep1": Bc * 256, "keep2": Bn * 256}[which]
        n = size - first if n is None else n
        out = torch.empty(max(n, 0), device=self.device)
        _lib.check(_lib.lib().dad_rng_draws(cfg, self._DRAWS[which], first, n, _lib.ptr(out), self._stream()),
                   "dad_rng_draws")
        return out

    def epoch_end(self):
        """DACPManager.update_class_quality_scores_epoch (I/utils.py:430-447), on device."""
        cfg = self.make_config(1, 1, 1, 1, self.view.WARMUP_EPOCHS)
        st = self._state_struct(0)
        _lib.check(_lib.lib().dad_epoch_end(cfg, st, self._stream()), "dad_epoch_end")

