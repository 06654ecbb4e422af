"""ctypes binding of the C ABI in include/dad.h (libdad_hip.so).

The structures below mirror dad.h field for field.  Loading fails loudly: there is no
Python or PyTorch fallback for any operator of the step.
"""
import ctypes
import os

from . import _build

c_float_p = ctypes.POINTER(ctypes.c_float)

DAD_ABI_VERSION = 7        # dad.h DAD_ABI_VERSION this binding mirrors
DAD_NPARAM = 256 * 768 + 256 + 4 * 256 + 4
DAD_GRAD_EXTRA = 16
DAD_GRAD_FLOATS = DAD_NPARAM + DAD_GRAD_EXTRA
DAD_DACP_FLOATS = 20
DAD_TAIL_HDR = 64
DAD_MAX_BATCH = 1024
PREC_FP32, PREC_BF16, PREC_FP16 = 0, 1, 2
DRAW_WEAK, DRAW_STRONG, DRAW_FEAT_KEEP, DRAW_TSTART, DRAW_KEEP1, DRAW_KEEP2 = range(1, 7)
RNG_EXPLICIT, RNG_COUNTER = 0, 1
PREP_CLEAN, PREP_NOISY = 1, 2     # dad.h DAD_PREP_* (dad_step_backward_ahead_split / dad_step_prepare_rows)

# tail header slots (dad.h DAD_T_*)
T_TOTAL, T_CE, T_KL, T_ECDA, T_SCL, T_MSUM, T_CLIPNORM, T_CLIPCOEF = range(8)
T_W, T_TAU_BEFORE, T_TAU_AFTER, T_FLOORED, T_ECDA_TERM, T_ECDA_GATE = 8, 12, 16, 20, 24, 28
T_KL_ON, T_ECDA_ON, T_RANGE, T_TAU_HAT = 32, 33, 34, 40
RANGE_NONFINITE, RANGE_POOL_TIMEOUT = 1, 2   # bits of the T_RANGE word (dad.h DAD_RANGE_*)


def tail_floats(bn):
    return DAD_TAIL_HDR + bn * 7


class DadConfig(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int32), ("T", ctypes.c_int32), ("Bn", ctypes.c_int32), ("Tn", ctypes.c_int32),
        ("precision", ctypes.c_int32), ("rng_mode", ctypes.c_int32),
        ("seed", ctypes.c_uint64), ("counter", ctypes.c_uint64),
        ("warmup", ctypes.c_int32), ("use_dacp", ctypes.c_int32), ("ecda_on", ctypes.c_int32),
        ("use_entropy", ctypes.c_int32), ("class_aware", ctypes.c_int32), ("dp_world", ctypes.c_int32),
        ("w_kl", ctypes.c_float), ("w_ecda", ctypes.c_float), ("dacp_gamma", ctypes.c_float),
        ("dacp_k", ctypes.c_float), ("dacp_lambda", ctypes.c_float), ("dacp_alpha", ctypes.c_float),
        ("dacp_one_m_alpha", ctypes.c_float), ("fixed_thr", ctypes.c_float),
        ("ecda_att_lambda", ctypes.c_float), ("ecda_gamma", ctypes.c_float), ("ecda_delta", ctypes.c_float),
        ("ls_eps", ctypes.c_float), ("p_drop", ctypes.c_float), ("drop_scale", ctypes.c_float),
        ("feat_p", ctypes.c_float), ("weak_std", ctypes.c_float), ("strong_std", ctypes.c_float),
        ("mask_len", ctypes.c_int32), ("start_hi", ctypes.c_int32), ("clip", ctypes.c_int32),
        ("max_norm", ctypes.c_float), ("lr_step_size", ctypes.c_float), ("bc2_sqrt", ctypes.c_float),
        ("beta1", ctypes.c_float), ("one_m_beta1", ctypes.c_float), ("beta2", ctypes.c_float),
        ("one_m_beta2", ctypes.c_float), ("adam_eps", ctypes.c_float), ("weight_decay", ctypes.c_float),
        ("ema_m", ctypes.c_float), ("ema_one_m", ctypes.c_float),
        ("dacp_beta", ctypes.c_float), ("dacp_one_m_beta", ctypes.c_float),
        ("splits", ctypes.c_int32), ("prepped", ctypes.c_int32), ("reserved", ctypes.c_int32 * 4),
    ]


class DadBatch(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in
                ("xc", "mc", "yc", "xn", "mn", "nw", "ns", "u", "start", "keep1", "keep2",
                 "rowc", "lenc", "rown", "lenn")]


class DadState(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in
                ("student", "teacher", "exp_avg", "exp_avg_sq", "grad", "w1bf_student", "w1bf_teacher",
                 "dacp", "tail", "emb", "logits", "losses")]


# exported symbols (must match include/dad.h); tests check every one is present
EXPORTS = {
    "dad_abi_version": (ctypes.c_int, []),
    "dad_param_count": (ctypes.c_size_t, []),
    "dad_workspace_bytes": (ctypes.c_int, [ctypes.POINTER(DadConfig), ctypes.POINTER(ctypes.c_size_t)]),
    "dad_error_string": (ctypes.c_char_p, [ctypes.c_int]),
    "dad_encoder_ws_plan": (ctypes.c_int, [ctypes.POINTER(DadConfig), ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                           ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "dad_encoder_ws_jobs": (ctypes.c_int, [ctypes.POINTER(DadConfig), ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                            ctypes.c_int]),
    "dad_step_compute": (ctypes.c_int, [ctypes.POINTER(DadConfig), ctypes.POINTER(DadBatch),
                                        ctypes.POINTER(DadState), ctypes.c_void_p, ctypes.c_void_p]),
    "dad_step_encode": (ctypes.c_int, [ctypes.POINTER(DadConfig), ctypes.POINTER(DadBatch),
                                       ctypes.POINTER(DadState), ctypes.c_void_p, ctypes.c_void_p]),
    "dad_step_backward": (ctypes.c_int, [ctypes.POINTER(DadConfig), ctypes.POINTER(DadBatch),
                                         ctypes.POINTER(DadState), ctypes.c_void_p, ctypes.c_void_p]),
    "dad_step_backward_ahead": (ctypes.c_int, [ctypes.POINTER(DadConfig), ctypes.POINTER(DadBatch),
                                               ctypes.POINTER(DadState), ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.POINTER(DadConfig), ctypes.POINTER(DadBatch),
                                               ctypes.POINTER(ctypes.c_int)]),
    "dad_step_backward_ahead_split": (ctypes.c_int, [ctypes.POINTER(DadConfig), ctypes.POINTER(DadBatch),
                                                     ctypes.POINTER(DadState), ctypes.c_void_p, ctypes.c_void_p,
                                                     ctypes.POINTER(DadConfig), ctypes.POINTER(DadBatch), ctypes.c_int,
                                                     ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "dad_step_prepare_rows": (ctypes.c_int, [ctypes.POINTER(DadConfig), ctypes.POINTER(DadBatch), ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_int]),
    "dad_step_apply": (ctypes.c_int, [ctypes.POINTER(DadConfig), ctypes.POINTER(DadState),
                                      ctypes.c_void_p, ctypes.c_void_p]),
    "dad_step": (ctypes.c_int, [ctypes.POINTER(DadConfig), ctypes.POINTER(DadBatch), ctypes.POINTER(DadState),
                                ctypes.c_void_p, ctypes.c_void_p]),
    "dad_step_commit": (ctypes.c_int, [ctypes.POINTER(DadConfig), ctypes.POINTER(DadState),
                                       ctypes.c_void_p, ctypes.c_void_p]),
    "dad_epoch_end": (ctypes.c_int, [ctypes.POINTER(DadConfig), ctypes.POINTER(DadState), ctypes.c_void_p]),
    "dad_refresh_shadow": (ctypes.c_int, [ctypes.POINTER(DadState), ctypes.c_int, ctypes.c_void_p]),
    "dad_teacher_ema": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_float,
                                       ctypes.c_float, ctypes.c_void_p]),
    "dad_encoder_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int, ctypes.c_int]),
    "dad_encoder_forward": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                           ctypes.c_void_p, ctypes.c_void_p]),
    "dad_encoder_backward": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "dad_collate": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                   ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "dad_collate_index": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "dad_collate_index_epoch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                               ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_void_p]),
    "dad_predict_head": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p]),
    "dad_augment": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_float, ctypes.c_float, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "dad_certainty_scores": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p]),
    "dad_dacp_mask": (ctypes.c_int, [ctypes.POINTER(DadConfig), ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p]),
    "dad_ecda_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int, ctypes.c_int]),
    "dad_ecda_loss": (ctypes.c_int, [ctypes.POINTER(DadConfig), ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                     ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "dad_rng_draws": (ctypes.c_int, [ctypes.POINTER(DadConfig), ctypes.c_int, ctypes.c_uint64, ctypes.c_size_t,
                                     ctypes.c_void_p, ctypes.c_void_p]),
    "dad_timing_start": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "dad_timing_kernels": (ctypes.c_int, [ctypes.c_uint]),
    "dad_timing_reset": (ctypes.c_int, []),
    "dad_timing_stop": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    "dad_comm_unique_id_bytes": (ctypes.c_int, []),
    "dad_comm_get_unique_id": (ctypes.c_int, [ctypes.c_void_p]),
    "dad_comm_init": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_void_p, ctypes.c_int]),
    "dad_comm_allreduce_grad": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(DadState), ctypes.c_void_p]),
    "dad_comm_count": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
    "dad_comm_allreduce_f32": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "dad_comm_destroy": (ctypes.c_int, [ctypes.c_void_p]),
}

# per-kernel timing slots (dad.h DAD_TK_*)
TK_NAMES = ["encode", "pool", "tail", "wgrad", "reduce", "optim"]

_LIB = None


class DadError(RuntimeError):
    pass


def lib():
    """Load libdad_hip.so (in-tree).  Raises if it is missing: build it with _build.build()."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = _build.lib_path(os.environ.get("DAD_LIB_VARIANT") or None)
    if not os.path.exists(path):
        raise DadError("libdad_hip.so not built (%s); run __graft_entry__.build() or "
                       "python -m <pkg>._build" % path)
    L = ctypes.CDLL(path)
    if not hasattr(L, "dad_abi_version"):
        raise DadError("%s predates ABI 6 (no dad_abi_version): rebuild it (__graft_entry__.build())" % path)
    for name, (res, args) in EXPORTS.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    ver = L.dad_abi_version()
    if ver != DAD_ABI_VERSION:
        raise DadError("%s was built for ABI %d, this binding needs ABI %d: rebuild it (__graft_entry__.build())"
                       % (path, ver, DAD_ABI_VERSION))
    _LIB = L
    return L


def check(rc, what=""):
    if rc != 0:
        msg = lib().dad_error_string(rc)
        raise DadError("%s failed: %s (%d)" % (what, msg.decode() if msg else "?", rc))


def ptr(t):
    """Device pointer of a tensor (or None)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class KernelTimer:
    """dad_timing_start / dad_timing_stop: mean duration (ms) per kernel of the fused step over
    every `every`-th step while active.  `stop()` returns {name: (mean_ms, n_steps)}."""

    def __init__(self, every=4, max_steps=256, kernels=None):
        """kernels: names (TK_NAMES) to time, default all; each recorded event costs stream time.
        One timer at a time: dad_timing_start refuses (DadError) while another is active."""
        check(lib().dad_timing_start(int(every), int(max_steps)), "dad_timing_start")
        if kernels is not None:
            mask = 0
            for k in kernels:
                mask |= 1 << TK_NAMES.index(k)
            check(lib().dad_timing_kernels(mask), "dad_timing_kernels")
        self.active = True

    def reset(self):
        """dad_timing_reset: the steps so far (a warm-up) are not counted; the events stay created."""
        check(lib().dad_timing_reset(), "dad_timing_reset")

    def stop(self):
        n = len(TK_NAMES)
        ms = (ctypes.c_double * n)()
        cnt = (ctypes.c_int * n)()
        self.active = False
        check(lib().dad_timing_stop(ms, cnt, n), "dad_timing_stop")
        return {TK_NAMES[k]: (ms[k] / cnt[k], cnt[k]) for k in range(n) if cnt[k] > 0}
