"""Late-bound view of the reference's config module(s) -> the C-ABI `dad_config` POD.

The reference keeps hyper-parameters as module constants (I/config.py, C/config_casia.py,
E/config_emodb.py) and reads them at CALL time (I/utils.py:410,567 re-import config inside
the functions; the ablation runners `setattr` them between runs,
I/run_granular_ablations.py:25-30).  `ConfigView` therefore reads its source on every
step; `dad_config_for()` converts the values to the float32 scalars torch would use for
the python-float operands (e.g. `(1 - alpha) * t` multiplies by float32(1 - alpha)).
"""
import math
import types

import numpy as np

from . import _lib

F32 = np.float32

_COMMON = dict(
    INPUT_DIM=768, HIDDEN_DIM=256, NUM_CLASSES=4, DROPOUT_RATE=0.1, EMA_MOMENTUM=0.995,
    WARMUP_EPOCHS=30, ECDA_START_EPOCH=30, DACP_SENSITIVITY_K=10.0,
    DACP_QUANTILE_START=0.4, DACP_QUANTILE_END=0.8, DACP_THRESHOLD_SMOOTHING_ALPHA=0.9,
    USE_ENTROPY_IN_SCORE=True, USE_CLASS_AWARE_MMD=True, ECDA_CLASS_ATTENTION_LAMBDA=1.0,
    WEIGHT_CONSISTENCY=1.0, EPOCHS=500, WEIGHT_DECAY=1e-5, USE_LABEL_SMOOTHING=True,
    LABEL_SMOOTHING_FACTOR=0.05, WEAK_NOISE_STD=0.01, STRONG_NOISE_STD=0.05,
    TEMPORAL_MASK_RATIO=0.1, PROGRESSIVE_TRAINING=True, INITIAL_CONSISTENCY_WEIGHT=0.1,
    FINAL_CONSISTENCY_WEIGHT=0.3, WEIGHT_RAMP_EPOCHS=30, GRADIENT_CLIPPING=True,
    MAX_GRAD_NORM=1.0, USE_DACP=True, USE_ECDA=True, LEARNING_RATE_SCHEDULER="cosine",
    ANCHOR_STD_K=1.5, BATCH_SIZE=64,
)
# per-dataset defaults (I/config.py:60-123, C/config_casia.py:63-126, E/config_emodb.py:63-126)
FLAVOR_DEFAULTS = {
    "iemocap": dict(_COMMON, DACP_QUALITY_SMOOTHING_BETA=0.9, DACP_CALIBRATION_STRENGTH_LAMBDA=0.9,
                    FIXED_CONFIDENCE_THRESHOLD=0.9, ECDA_COMPACTNESS_WEIGHT_GAMMA=0.1,
                    ECDA_REPULSION_WEIGHT_DELTA=0.1, WEIGHT_ECDA=0.3, LEARNING_RATE=5e-4),
    "casia": dict(_COMMON, DACP_QUALITY_SMOOTHING_BETA=0.9, DACP_CALIBRATION_STRENGTH_LAMBDA=0.1,
                  USE_DACP=False, USE_ECDA=False, FIXED_CONFIDENCE_THRESHOLD=0.75,
                  ECDA_COMPACTNESS_WEIGHT_GAMMA=0.05, ECDA_REPULSION_WEIGHT_DELTA=0.05,
                  WEIGHT_ECDA=0.35, LEARNING_RATE=5e-4),
    "emodb": dict(_COMMON, DACP_QUALITY_SMOOTHING_BETA=0.8, DACP_CALIBRATION_STRENGTH_LAMBDA=0.3,
                  FIXED_CONFIDENCE_THRESHOLD=0.75, ECDA_COMPACTNESS_WEIGHT_GAMMA=0.1,
                  ECDA_REPULSION_WEIGHT_DELTA=0.1, WEIGHT_ECDA=0.1, LEARNING_RATE=5e-3),
}
_MODULE_FLAVOR = {"config": "iemocap", "config_casia": "casia", "config_emodb": "emodb"}


_MISSING = object()


class ConfigView:
    """Read-through view of a config source (module, dict or object) with dataset defaults.

    `flavor` selects which ablation switches the dataset's trainer honours (see
    `effective_switches`); it is inferred from the module name when not given.
    """

    def __init__(self, source=None, flavor=None, **overrides):
        if flavor is None:
            name = getattr(source, "__name__", "") if isinstance(source, types.ModuleType) else ""
            flavor = _MODULE_FLAVOR.get(name.split(".")[-1], "iemocap")
        if flavor not in FLAVOR_DEFAULTS:
            raise ValueError("unknown flavor %r" % flavor)
        self.flavor = flavor
        self.source = source
        self.overrides = dict(overrides)

    def __getattr__(self, name):
        # called for every config read of every step (dad_config_for reads ~40): one dict fetch
        # per source, no hasattr + getattr pairs
        if name[:1] == "_" or name in ("flavor", "source", "overrides"):
            raise AttributeError(name)
        d = self.__dict__
        ov = d.get("overrides")
        if ov and name in ov:
            return ov[name]
        src = d.get("source")
        if src is not None:
            if type(src) is dict or isinstance(src, dict):
                if name in src:
                    return src[name]
            else:
                v = getattr(src, name, _MISSING)
                if v is not _MISSING:
                    return v
        fl = d.get("flavor")
        if fl is not None:
            dd = FLAVOR_DEFAULTS[fl]
            if name in dd:
                return dd[name]
        raise AttributeError(name)

    def effective_switches(self):
        """(use_dacp, use_ecda, use_entropy, class_aware) as each trainer applies them.

        IEMOCAP honours all four switches; CASIA has no entropy / class-aware switch
        (C/utils.py:412-422, 572-626); EMODB also ignores USE_DACP (E/train_emodb.py:419)
        and USE_ECDA (E/train_emodb.py:437).
        """
        fl = self.flavor
        use_dacp = bool(self.USE_DACP) if fl != "emodb" else True
        use_ecda = bool(self.USE_ECDA) if fl != "emodb" else True
        use_entropy = bool(self.USE_ENTROPY_IN_SCORE) if fl == "iemocap" else True
        class_aware = bool(self.USE_CLASS_AWARE_MMD) if fl == "iemocap" else True
        return use_dacp, use_ecda, use_entropy, class_aware

    def loss_weights(self, epoch):
        """`update_loss_weights` (I/train.py:380-395) -> (w_kl, w_ecda, warmup)."""
        if epoch < self.WARMUP_EPOCHS:
            return 0.0, 0.0, True
        if self.PROGRESSIVE_TRAINING:
            init_w, final_w = self.INITIAL_CONSISTENCY_WEIGHT, self.FINAL_CONSISTENCY_WEIGHT
            prog = min(1.0, (epoch - self.WARMUP_EPOCHS) / self.WEIGHT_RAMP_EPOCHS)
            w_kl = init_w + (final_w - init_w) * prog
        else:
            w_kl = self.WEIGHT_CONSISTENCY
        if epoch >= self.ECDA_START_EPOCH:
            w_ecda = self.WEIGHT_ECDA * min(1.0, (epoch - self.ECDA_START_EPOCH) / self.WEIGHT_RAMP_EPOCHS)
        else:
            w_ecda = 0.0
        return w_kl, w_ecda, False

    def lr_at(self, epoch):
        """CosineAnnealingLR(T_max=EPOCHS) after `epoch` scheduler steps (I/train.py:363,519)."""
        if getattr(self, "LEARNING_RATE_SCHEDULER", "cosine") != "cosine":
            return self.LEARNING_RATE
        return self.LEARNING_RATE * (1 + math.cos(math.pi * epoch / self.EPOCHS)) / 2


def dad_config_for(view, Bc, Tc, Bn, Tn, epoch, adam_step, lr=None, precision=_lib.PREC_FP32,
                   rng_mode=_lib.RNG_COUNTER, seed=0, counter=0, dp_world=1, splits=0):
    """Fill a `dad_config` for one step. `adam_step` is the Adam step count AFTER this step.
    (The c_float fields round each Python float to nearest, as np.float32 would; only drop_scale
    is computed in float32 arithmetic, as nn.Dropout's 1/(1-p) is.)"""
    if view.INPUT_DIM != 768 or view.HIDDEN_DIM != 256 or view.NUM_CLASSES != 4:
        raise ValueError("the MI355X kernels are built for INPUT_DIM=768, HIDDEN_DIM=256, NUM_CLASSES=4")
    use_dacp, use_ecda, use_entropy, class_aware = view.effective_switches()
    w_kl, w_ecda, warm = view.loss_weights(epoch)
    if lr is None:
        lr = view.lr_at(epoch)
    c = _lib.DadConfig()
    c.B, c.T = int(Bc), int(Tc)
    c.Bn, c.Tn = (0, 0) if warm and Bn is None else (int(Bn), int(Tn))
    c.precision, c.rng_mode = int(precision), int(rng_mode)
    c.seed, c.counter = int(seed) & (2 ** 64 - 1), int(counter) & (2 ** 64 - 1)
    c.warmup = int(warm)
    c.use_dacp, c.use_entropy, c.class_aware = int(use_dacp), int(use_entropy), int(class_aware)
    c.ecda_on = int(use_ecda and w_ecda > 0)
    c.dp_world = int(dp_world)
    c.w_kl, c.w_ecda = w_kl, w_ecda
    gamma = view.DACP_QUANTILE_START + (view.DACP_QUANTILE_END - view.DACP_QUANTILE_START) * (epoch / view.EPOCHS)
    c.dacp_gamma = gamma
    a = view.DACP_THRESHOLD_SMOOTHING_ALPHA
    c.dacp_k, c.dacp_lambda = view.DACP_SENSITIVITY_K, view.DACP_CALIBRATION_STRENGTH_LAMBDA
    c.dacp_alpha, c.dacp_one_m_alpha = a, 1 - a
    c.fixed_thr = view.FIXED_CONFIDENCE_THRESHOLD
    c.ecda_att_lambda = view.ECDA_CLASS_ATTENTION_LAMBDA
    c.ecda_gamma, c.ecda_delta = view.ECDA_COMPACTNESS_WEIGHT_GAMMA, view.ECDA_REPULSION_WEIGHT_DELTA
    c.ls_eps = view.LABEL_SMOOTHING_FACTOR if view.USE_LABEL_SMOOTHING else 0.0
    p = view.DROPOUT_RATE
    c.p_drop = p
    c.drop_scale = F32(1.0) / F32(1 - p) if p < 1 else F32(0.0)
    c.feat_p = p                                   # DataAugmentation.dropout_rate (I/utils.py:325)
    c.weak_std, c.strong_std = view.WEAK_NOISE_STD, view.STRONG_NOISE_STD
    tn = c.Tn if c.Tn > 0 else 1
    mlen = int(tn * view.TEMPORAL_MASK_RATIO) if view.TEMPORAL_MASK_RATIO > 0 else 0
    c.mask_len = mlen
    c.start_hi = max(1, tn - mlen + 1)
    c.clip = int(bool(view.GRADIENT_CLIPPING))
    c.max_norm = view.MAX_GRAD_NORM
    b1, b2 = 0.9, 0.999
    c.lr_step_size = lr / (1 - b1 ** adam_step)
    c.bc2_sqrt = math.sqrt(1 - b2 ** adam_step)
    c.beta1, c.one_m_beta1, c.beta2, c.one_m_beta2 = b1, 1 - b1, b2, 1 - b2
    c.adam_eps, c.weight_decay = 1e-8, view.WEIGHT_DECAY
    m = view.EMA_MOMENTUM
    c.ema_m, c.ema_one_m = m, 1.0 - m
    beta = view.DACP_QUALITY_SMOOTHING_BETA
    c.dacp_beta, c.dacp_one_m_beta = beta, 1 - beta
    c.splits = int(splits)
    return c


# Every attribute dad_config_for (and the ConfigView methods it calls) reads: the key of
# ConfigCache.  tests/test_config_model_cpu.py records the attributes a dad_config_for call
# actually reads and checks that they are all here.
CONFIG_KEYS = (
    "INPUT_DIM", "HIDDEN_DIM", "NUM_CLASSES",
    "USE_DACP", "USE_ECDA", "USE_ENTROPY_IN_SCORE", "USE_CLASS_AWARE_MMD",
    "WARMUP_EPOCHS", "PROGRESSIVE_TRAINING", "INITIAL_CONSISTENCY_WEIGHT", "FINAL_CONSISTENCY_WEIGHT",
    "WEIGHT_RAMP_EPOCHS", "WEIGHT_CONSISTENCY", "ECDA_START_EPOCH", "WEIGHT_ECDA",
    "LEARNING_RATE_SCHEDULER", "LEARNING_RATE", "EPOCHS",
    "DACP_QUANTILE_START", "DACP_QUANTILE_END", "DACP_THRESHOLD_SMOOTHING_ALPHA", "DACP_SENSITIVITY_K",
    "DACP_CALIBRATION_STRENGTH_LAMBDA", "FIXED_CONFIDENCE_THRESHOLD", "ECDA_CLASS_ATTENTION_LAMBDA",
    "ECDA_COMPACTNESS_WEIGHT_GAMMA", "ECDA_REPULSION_WEIGHT_DELTA", "LABEL_SMOOTHING_FACTOR",
    "USE_LABEL_SMOOTHING", "DROPOUT_RATE", "WEAK_NOISE_STD", "STRONG_NOISE_STD", "TEMPORAL_MASK_RATIO",
    "GRADIENT_CLIPPING", "MAX_GRAD_NORM", "WEIGHT_DECAY", "EMA_MOMENTUM", "DACP_QUALITY_SMOOTHING_BETA",
)


def _view_values(view):
    """The CONFIG_KEYS values of a ConfigView in one pass (a sentinel for missing ones), or None
    for another view type (then nothing is cached)."""
    if type(view) is not ConfigView:
        return None
    d = view.__dict__
    ov = d.get("overrides") or {}
    src = d.get("source")
    dd = FLAVOR_DEFAULTS[d["flavor"]]
    out = []
    if src is None:
        for k in CONFIG_KEYS:
            out.append(ov[k] if k in ov else dd.get(k, _MISSING))
    elif isinstance(src, dict):
        for k in CONFIG_KEYS:
            out.append(ov[k] if k in ov else (src[k] if k in src else dd.get(k, _MISSING)))
    else:
        for k in CONFIG_KEYS:
            if k in ov:
                out.append(ov[k])
            else:
                v = getattr(src, k, _MISSING)
                out.append(v if v is not _MISSING else dd.get(k, _MISSING))
    return (d["flavor"],) + tuple(out)


class ConfigCache:
    """dad_config_for with its step-independent part cached: the config of a (view contents,
    geometry, epoch, lr, precision, RNG, world, splits) key is built once by dad_config_for, and
    each step copies it and sets only the Adam step's two scalars and the RNG counter, with
    dad_config_for's own expressions, so the result is byte-identical.  The key holds every value
    the view gives dad_config_for (CONFIG_KEYS, read in one pass each call), so a changed config
    value is a new key.  (dad_config_for reads ~40 view attributes and sets ~60 ctypes fields:
    ~20 us of host time per step, a third of DADStep.step's.)"""

    def __init__(self, max_entries=64):
        self._d = {}
        self._max = max_entries

    def config(self, view, Bc, Tc, Bn, Tn, epoch, adam_step, lr=None, precision=_lib.PREC_FP32,
               rng_mode=_lib.RNG_COUNTER, seed=0, counter=0, dp_world=1, splits=0):
        vals = _view_values(view)
        key = (vals, Bc, Tc, Bn, Tn, epoch, lr, int(precision), int(rng_mode), int(seed), int(dp_world), int(splits))
        try:
            hit = self._d.get(key) if vals is not None else None
        except TypeError:          # an unhashable config value: no caching
            vals = None
        if vals is None:
            return dad_config_for(view, Bc, Tc, Bn, Tn, epoch, adam_step, lr=lr, precision=precision,
                                  rng_mode=rng_mode, seed=seed, counter=counter, dp_world=dp_world, splits=splits)
        if hit is None:
            base = dad_config_for(view, Bc, Tc, Bn, Tn, epoch, 1, lr=lr, precision=precision, rng_mode=rng_mode,
                                  seed=seed, counter=0, dp_world=dp_world, splits=splits)
            lr_eff = lr if lr is not None else view.lr_at(epoch)
            if len(self._d) >= self._max:
                self._d.clear()
            hit = self._d[key] = (base, lr_eff)
        base, lr_eff = hit
        c = _lib.DadConfig.from_buffer_copy(base)
        c.counter = int(counter) & (2 ** 64 - 1)
        b1, b2 = 0.9, 0.999
        c.lr_step_size = lr_eff / (1 - b1 ** adam_step)
        c.bc2_sqrt = math.sqrt(1 - b2 ** adam_step)
        return c
