"""The reference's DAD helper types (I/utils.py:317-652) as drop-ins on the MI355X operators.

Trainer code that drives the helpers itself -- `train_step` (I/train.py:397-471) through the
shim's callers, anchor calibration (`DACPManager.calculate_certainty_scores`,
I/train.py:334,341), the epoch-end quality update (I/train.py:498-499) -- finds the same
classes, constructors, methods and fields here:

    DataAugmentation(weak_noise_std, strong_noise_std, dropout_rate, temporal_mask_ratio)
        .weak_augment(x) / .strong_augment(x) / ._apply_temporal_masking(x)      dad_augment
    DACPManager(num_classes, total_epochs, device)
        .calculate_certainty_scores(probs)  (static)                              dad_certainty_scores
        .calculate_mask(teacher_probs, epoch, calibrated_anchors)                 dad_dacp_mask
        .update_class_quality_scores_epoch(epoch_scores_per_class)
        .ema_thresholds, .class_quality_scores, .batch_scores_per_class
    ECDALoss()(clean_feats, noisy_feats, clean_labels, noisy_labels,
               noisy_mask, noisy_scores, class_weights_wce)                       dad_ecda_loss

Every operator is a HIP kernel behind the C ABI (include/dad.h), running the device
functions of the fused step; tensors must be on the GPU.  Config is read at call time
(`ConfigView`), as the reference re-imports `config` inside the functions
(I/utils.py:410,567).  Randomness: the reference draws from torch's global generator; here
the counter streams of (seed, call counter) -- the same streams the fused step uses -- or
explicit draws passed as keyword arguments (parity tests).
"""
import numpy as np
import torch

from . import _lib
from .config import ConfigView, dad_config_for


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _need_cuda(t, what):
    if not (torch.is_tensor(t) and t.is_cuda):
        raise RuntimeError("%s: the MI355X operators take GPU tensors (got %s)" % (
            what, t.device if torch.is_tensor(t) else type(t).__name__))


def _view(cfg):
    return cfg if isinstance(cfg, ConfigView) else ConfigView(cfg)


class DataAugmentation:
    """`DataAugmentation` (I/utils.py:317-375): teacher weak vs student strong augmentation."""

    def __init__(self, weak_noise_std=None, strong_noise_std=None, dropout_rate=None, temporal_mask_ratio=None,
                 cfg=None, seed=0):
        v = _view(cfg)
        self.weak_noise_std = weak_noise_std if weak_noise_std is not None else v.WEAK_NOISE_STD
        self.strong_noise_std = strong_noise_std if strong_noise_std is not None else v.STRONG_NOISE_STD
        self.dropout_rate = dropout_rate if dropout_rate is not None else v.DROPOUT_RATE
        self.temporal_mask_ratio = temporal_mask_ratio if temporal_mask_ratio is not None else v.TEMPORAL_MASK_RATIO
        self.seed = int(seed)
        self.counter = 0          # one counter value per augment call (the fused step: one per step)

    @staticmethod
    def _geometry(data):
        """(B, T, D) of the kernel's [B][T][D] view and whether temporal masking applies
        (I/utils.py:347,354,364: 2-D [T, D] and 3-D [B, T, D] data only)."""
        if data.dim() == 3:
            return data.shape[0], data.shape[1], data.shape[2], True
        if data.dim() == 2:
            return 1, data.shape[0], data.shape[1], True
        D = data.shape[-1] if data.dim() else 1
        return 1, max(1, data.numel() // max(D, 1)), D, False

    def _run(self, data, strong, noise=None, u=None, start=None, temporal=True):
        _need_cuda(data, "DataAugmentation")
        x = data.contiguous().float()
        B, T, D, masked = self._geometry(x)
        ratio = float(self.temporal_mask_ratio) if (strong and temporal and masked) else 0.0
        mlen = int(T * ratio) if ratio > 0 else 0        # I/utils.py:356,366
        p = float(self.dropout_rate) if strong else 0.0
        sd = float(self.strong_noise_std if strong else self.weak_noise_std)
        out = torch.empty_like(x)
        keep = []

        def dev(t, dtype):
            if t is None:
                return None
            t = torch.as_tensor(t).to(device=x.device, dtype=dtype).contiguous()
            keep.append(t)
            return t.data_ptr()
        _lib.check(_lib.lib().dad_augment(x.data_ptr(), B, T, D, int(strong), np.float32(sd), np.float32(p), mlen,
                                          self.seed, self.counter, dev(noise, torch.float32), dev(u, torch.float32),
                                          dev(start, torch.int64), out.data_ptr(), _stream(x)), "dad_augment")
        self.counter += 1
        return out.view(data.shape)

    def weak_augment(self, data, noise=None):
        """x + randn_like(x) * weak_noise_std (I/utils.py:328-331)."""
        return self._run(data, False, noise=noise)

    def strong_augment(self, data, noise=None, u=None, start=None):
        """noise, feature dropout (one [D] mask, no rescale), temporal masking (I/utils.py:333-375)."""
        return self._run(data, True, noise=noise, u=u, start=start)

    def _apply_temporal_masking(self, data, start=None):
        """Temporal masking alone (I/utils.py:352-375): no noise, no feature mask."""
        keep_p, keep_sd = self.dropout_rate, self.strong_noise_std
        self.dropout_rate, self.strong_noise_std = 0.0, 0.0
        try:
            zero = torch.zeros(data.numel(), device=data.device)
            return self._run(data, True, noise=zero, start=start)
        finally:
            self.dropout_rate, self.strong_noise_std = keep_p, keep_sd


class _ScoreLog:
    """`batch_scores_per_class`: the per-class certainty scores collected by calculate_mask
    since the last epoch update (I/utils.py:503-505).  Kept on the device (one (score, pred)
    pair of tensors per call, no host sync); read as the reference's list of lists."""

    def __init__(self, num_classes):
        self.num_classes = num_classes
        self.parts = []

    def lists(self):
        out = [[] for _ in range(self.num_classes)]
        for s, p in self.parts:
            s, p = s.cpu().numpy(), p.cpu().numpy()
            for c in range(self.num_classes):
                out[c].extend(s[p == c])
        return out

    def __len__(self):
        return self.num_classes

    def __getitem__(self, c):
        return self.lists()[c]

    def __iter__(self):
        return iter(self.lists())


class DACPManager:
    """`DACPManager` (I/utils.py:379-507): certainty scores, per-class dynamic thresholds, mask."""

    def __init__(self, num_classes, total_epochs, device, cfg=None):
        if num_classes != 4:
            raise ValueError("the MI355X kernels are built for NUM_CLASSES=4")
        self.num_classes = num_classes
        self.total_epochs = total_epochs
        self.device = torch.device(device)
        self.view = _view(cfg)
        # the 20-float device state of the fused step: tau | Q | epoch sums | counts | anchors
        self.state = torch.zeros(_lib.DAD_DACP_FLOATS, device=self.device)
        self.state[0:4] = 0.5     # ema_thresholds (I/utils.py:395)
        self.state[4:8] = 0.5     # class_quality_scores (I/utils.py:391)
        self._log = _ScoreLog(num_classes)

    @property
    def ema_thresholds(self):
        return self.state[0:4]

    @ema_thresholds.setter
    def ema_thresholds(self, v):
        self.state[0:4] = torch.as_tensor(v, dtype=torch.float32).to(self.device)

    @property
    def class_quality_scores(self):
        return self.state[4:8]

    @class_quality_scores.setter
    def class_quality_scores(self, v):
        self.state[4:8] = torch.as_tensor(v, dtype=torch.float32).to(self.device)

    @property
    def batch_scores_per_class(self):
        return self._log

    @batch_scores_per_class.setter
    def batch_scores_per_class(self, v):
        if isinstance(v, _ScoreLog):
            self._log = v
            return
        self._log = _ScoreLog(self.num_classes)       # reset to empty lists (I/utils.py:447)
        self.state[8:16] = 0.0
        if any(len(x) for x in v):
            raise ValueError("batch_scores_per_class can only be reset to empty lists")

    @staticmethod
    def calculate_certainty_scores(probs, cfg=None):
        """(scores [B], preds [B]) of teacher probabilities (I/utils.py:400-428)."""
        _need_cuda(probs, "calculate_certainty_scores")
        q = probs.contiguous().float()
        if q.dim() != 2 or q.shape[1] != 4:
            raise ValueError("probs must be [B, 4]")
        v = _view(cfg)
        use_entropy = v.effective_switches()[2]
        B = q.shape[0]
        s = torch.empty(B, device=q.device)
        p = torch.empty(B, dtype=torch.int64, device=q.device)
        _lib.check(_lib.lib().dad_certainty_scores(q.data_ptr(), B, int(use_entropy), s.data_ptr(), p.data_ptr(),
                                                   _stream(q)), "dad_certainty_scores")
        return s, p

    def _config(self, Bn, epoch):
        c = dad_config_for(self.view, 1, 1, Bn, 1, epoch, 1)
        c.use_dacp = 1
        c.use_entropy = int(self.view.effective_switches()[2])
        # gamma_e = start + (end - start) * epoch / total_epochs (I/utils.py:472-473)
        v = self.view
        c.dacp_gamma = np.float32(v.DACP_QUANTILE_START + (v.DACP_QUANTILE_END - v.DACP_QUANTILE_START)
                                  * (epoch / self.total_epochs))
        return c

    def calculate_mask(self, teacher_probs, epoch, calibrated_anchors):
        """(mask bool [B], certainty_scores [B], class_weights_wce [C]) (I/utils.py:449-507);
        updates ema_thresholds and collects the scores for the epoch update."""
        _need_cuda(teacher_probs, "calculate_mask")
        q = teacher_probs.contiguous().float()
        Bn = q.shape[0]
        if calibrated_anchors is None:        # the reference crashes here (I/utils.py:491: None.to)
            raise AttributeError("'NoneType' object has no attribute 'to'")
        self.state[16:20] = torch.as_tensor(calibrated_anchors, dtype=torch.float32).to(self.device)
        mask = torch.empty(Bn, dtype=torch.uint8, device=q.device)
        s = torch.empty(Bn, device=q.device)
        p = torch.empty(Bn, dtype=torch.int64, device=q.device)
        w = torch.empty(4, device=q.device)
        _lib.check(_lib.lib().dad_dacp_mask(self._config(Bn, epoch), q.data_ptr(), Bn, self.state.data_ptr(),
                                            mask.data_ptr(), s.data_ptr(), p.data_ptr(), w.data_ptr(), _stream(q)),
                   "dad_dacp_mask")
        self._log.parts.append((s, p))
        return mask.bool(), s, w

    def update_class_quality_scores_epoch(self, epoch_scores_per_class):
        """Q <- beta Q + (1 - beta) mean(epoch scores per class) (I/utils.py:430-447)."""
        beta = np.float32(self.view.DACP_QUALITY_SMOOTHING_BETA)
        if epoch_scores_per_class is self._log:
            # the device sums and counts calculate_mask collected (the fused step's epoch end)
            _lib.check(_lib.lib().dad_epoch_end(self._epoch_cfg(beta), self._state_struct(), _stream(self.state)),
                       "dad_epoch_end")
        else:
            Q = self.state[4:8].cpu().numpy()
            cur = np.array([np.mean(s) if len(s) > 0 else Q[i] for i, s in enumerate(epoch_scores_per_class)],
                           np.float32)
            q_new = beta * torch.from_numpy(Q) + (np.float32(1) - beta) * torch.from_numpy(cur)
            self.state[4:8] = q_new.to(self.device)
            self.state[8:16] = 0.0
        self._log = _ScoreLog(self.num_classes)

    def _epoch_cfg(self, beta):
        c = _lib.DadConfig()
        c.dacp_beta, c.dacp_one_m_beta = beta, np.float32(1) - beta
        return c

    def _state_struct(self):
        st = _lib.DadState()
        st.dacp = self.state.data_ptr()
        return st


class _EcdaFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, clean, noisy, loss, gclean, gnoisy):
        ctx.save_for_backward(gclean, gnoisy)
        return loss.clone()

    @staticmethod
    def backward(ctx, g):
        gc, gn = ctx.saved_tensors
        return gc * g, gn * g, None, None, None


class ECDALoss(torch.nn.Module):
    """`ECDALoss` (I/utils.py:510-652): class-aware attention-weighted MMD + compactness +
    repulsion (or the global-MMD ablation), differentiable w.r.t. both embedding sets."""

    def __init__(self, kernel_type="rbf", kernel_mul=2.0, kernel_num=5, cfg=None):
        super().__init__()
        if kernel_type != "rbf" or kernel_mul != 2.0 or kernel_num != 5:
            raise ValueError("the ECDA kernels implement the reference's rbf kernel, kernel_mul=2, kernel_num=5")
        self.kernel_type, self.kernel_mul, self.kernel_num = kernel_type, kernel_mul, kernel_num
        self.view = _view(cfg)

    def forward(self, clean_feats, noisy_feats, clean_labels, noisy_labels, noisy_mask, noisy_scores,
                class_weights_wce):
        for t, n in ((clean_feats, "clean_feats"), (noisy_feats, "noisy_feats")):
            _need_cuda(t, "ECDALoss " + n)
        dev = clean_feats.device
        v = self.view
        if noisy_mask.dtype != torch.bool:       # confidence scores re-cast (I/utils.py:573-576)
            noisy_mask = noisy_mask > v.FIXED_CONFIDENCE_THRESHOLD
        w = class_weights_wce.to(dev, torch.float32).contiguous()
        B, Bn = clean_feats.shape[0], noisy_feats.shape[0]
        if w.numel() != 4:
            # the fixed-threshold branch passes ones(Bn) (I/train.py:420): unit class attention
            if w.numel() != Bn or not bool((w == 1).all()):
                raise NotImplementedError("class_weights_wce must be DACP's [4] weights or ones(Bn)")
        ec = clean_feats.detach().contiguous().float()
        en = noisy_feats.detach().contiguous().float()
        yc = clean_labels.to(dev, torch.int64).contiguous()
        yn = noisy_labels.to(dev, torch.int64).contiguous()
        m = noisy_mask.to(dev).contiguous().view(torch.uint8)
        sc = noisy_scores.detach().to(dev, torch.float32).contiguous()
        c = dad_config_for(v, 1, 1, 1, 1, v.WARMUP_EPOCHS, 1)
        c.class_aware = int(v.effective_switches()[3])
        loss = torch.empty((), device=dev)
        gc = torch.empty_like(ec)
        gn = torch.empty_like(en)
        ws = torch.empty(int(_lib.lib().dad_ecda_workspace_bytes(B, Bn)), dtype=torch.uint8, device=dev)
        _lib.check(_lib.lib().dad_ecda_loss(c, ec.data_ptr(), B, en.data_ptr(), Bn, yc.data_ptr(), yn.data_ptr(),
                                            m.data_ptr(), sc.data_ptr(), w.data_ptr(), w.numel(), loss.data_ptr(),
                                            gc.data_ptr(), gn.data_ptr(), ws.data_ptr(), _stream(ec)),
                   "dad_ecda_loss")
        return _EcdaFn.apply(clean_feats, noisy_feats, loss, gc, gn)
