"""CPU restatement of the reference DAD train step (TEST INFRASTRUCTURE ONLY).

This is the parity oracle: a NumPy restatement of the reference's hot path with a
hand-derived (analytic) backward.  It is pinned against golden vectors produced by
running the reference itself (tests/golden/gen_golden.py, fixtures tests/golden/*.npz).
Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg use it,
and only as the checker / the timed CPU baseline; the product package never imports it.

All references are to /root/reference; ``I/`` = IEMOCAP/DAD-train-IEMOCAP/,
``C/`` = CASIA/DAD-train-CASIA/, ``E/`` = EMODB/DAD-train-EMODB/.

Numerics: the big contractions run in float32 (like the reference's fp32 addmm);
the small loss tail runs in float64 and its outputs are rounded to float32, except
the DACP threshold path which mirrors torch's float32 op order (quantile, EMA) since
the mask comparison ``s >= tau`` is a discrete decision.
"""
import math

import numpy as np

F32 = np.float32


# --------------------------------------------------------------------------- config

# Defaults of the three config modules (I/config.py, C/config_casia.py, E/config_emodb.py).
_COMMON = dict(
    INPUT_DIM=768, HIDDEN_DIM=256, NUM_CLASSES=4, DROPOUT_RATE=0.1, EMA_MOMENTUM=0.995,
    WARMUP_EPOCHS=30, ECDA_START_EPOCH=30, DACP_SENSITIVITY_K=10.0,
    DACP_QUANTILE_START=0.4, DACP_QUANTILE_END=0.8, DACP_THRESHOLD_SMOOTHING_ALPHA=0.9,
    USE_ENTROPY_IN_SCORE=True, USE_CLASS_AWARE_MMD=True, ECDA_CLASS_ATTENTION_LAMBDA=1.0,
    WEIGHT_CONSISTENCY=1.0, EPOCHS=500, WEIGHT_DECAY=1e-5, USE_LABEL_SMOOTHING=True,
    LABEL_SMOOTHING_FACTOR=0.05, WEAK_NOISE_STD=0.01, STRONG_NOISE_STD=0.05,
    TEMPORAL_MASK_RATIO=0.1, PROGRESSIVE_TRAINING=True, INITIAL_CONSISTENCY_WEIGHT=0.1,
    FINAL_CONSISTENCY_WEIGHT=0.3, WEIGHT_RAMP_EPOCHS=30, GRADIENT_CLIPPING=True,
    MAX_GRAD_NORM=1.0, USE_DACP=True, USE_ECDA=True,
)
FLAVOR_DEFAULTS = {
    # I/config.py:70-105
    "iemocap": dict(_COMMON, DACP_QUALITY_SMOOTHING_BETA=0.9, DACP_CALIBRATION_STRENGTH_LAMBDA=0.9,
                    FIXED_CONFIDENCE_THRESHOLD=0.9, ECDA_COMPACTNESS_WEIGHT_GAMMA=0.1,
                    ECDA_REPULSION_WEIGHT_DELTA=0.1, WEIGHT_ECDA=0.3, LEARNING_RATE=5e-4),
    # C/config_casia.py:72-112
    "casia": dict(_COMMON, DACP_QUALITY_SMOOTHING_BETA=0.9, DACP_CALIBRATION_STRENGTH_LAMBDA=0.1,
                  USE_DACP=False, USE_ECDA=False, FIXED_CONFIDENCE_THRESHOLD=0.75,
                  ECDA_COMPACTNESS_WEIGHT_GAMMA=0.05, ECDA_REPULSION_WEIGHT_DELTA=0.05,
                  WEIGHT_ECDA=0.35, LEARNING_RATE=5e-4),
    # E/config_emodb.py:72-112
    "emodb": dict(_COMMON, DACP_QUALITY_SMOOTHING_BETA=0.8, DACP_CALIBRATION_STRENGTH_LAMBDA=0.3,
                  FIXED_CONFIDENCE_THRESHOLD=0.75, ECDA_COMPACTNESS_WEIGHT_GAMMA=0.1,
                  ECDA_REPULSION_WEIGHT_DELTA=0.1, WEIGHT_ECDA=0.1, LEARNING_RATE=5e-3),
}


def make_cfg(flavor, **overrides):
    c = dict(FLAVOR_DEFAULTS[flavor])
    c.update(overrides)
    c["flavor"] = flavor
    return c


def effective_switches(cfg):
    """Which ablation switches a dataset's trainer honours.

    IEMOCAP honours all four; CASIA has no entropy/class-aware switches (C/utils.py:412-422,
    572-626); EMODB additionally ignores USE_DACP (E/train_emodb.py:419) and USE_ECDA
    (E/train_emodb.py:437: ECDA gated by weight only).
    """
    fl = cfg["flavor"]
    use_dacp = cfg["USE_DACP"] if fl != "emodb" else True
    use_ecda = cfg["USE_ECDA"] if fl != "emodb" else True
    use_entropy = cfg["USE_ENTROPY_IN_SCORE"] if fl == "iemocap" else True
    class_aware = cfg["USE_CLASS_AWARE_MMD"] if fl == "iemocap" else True
    return use_dacp, use_ecda, use_entropy, class_aware


def loss_weights(cfg, epoch):
    """`update_loss_weights` (I/train.py:380-395) -> (w_kl, w_ecda, warmup)."""
    if epoch < cfg["WARMUP_EPOCHS"]:
        return 0.0, 0.0, True
    init_w = cfg["INITIAL_CONSISTENCY_WEIGHT"] if cfg["PROGRESSIVE_TRAINING"] else cfg["WEIGHT_CONSISTENCY"]
    final_w = cfg["FINAL_CONSISTENCY_WEIGHT"] if cfg["PROGRESSIVE_TRAINING"] else cfg["WEIGHT_CONSISTENCY"]
    if cfg["PROGRESSIVE_TRAINING"]:
        prog = min(1.0, (epoch - cfg["WARMUP_EPOCHS"]) / cfg["WEIGHT_RAMP_EPOCHS"])
        w_kl = init_w + (final_w - init_w) * prog
    else:
        w_kl = cfg["WEIGHT_CONSISTENCY"]
    if epoch >= cfg["ECDA_START_EPOCH"]:
        w_ecda = cfg["WEIGHT_ECDA"] * min(1.0, (epoch - cfg["ECDA_START_EPOCH"]) / cfg["WEIGHT_RAMP_EPOCHS"])
    else:
        w_ecda = 0.0
    return w_kl, w_ecda, False


def cosine_lr(cfg, epoch):
    """CosineAnnealingLR(T_max=EPOCHS) value after `epoch` scheduler steps (I/train.py:363,519)."""
    return cfg["LEARNING_RATE"] * (1 + math.cos(math.pi * epoch / cfg["EPOCHS"])) / 2


# ------------------------------------------------------------------ small primitives

def softmax(z):
    z = np.asarray(z, np.float64)
    m = z.max(axis=1, keepdims=True)
    e = np.exp(z - m)
    return e / e.sum(axis=1, keepdims=True)


def log_softmax(z):
    z = np.asarray(z, np.float64)
    m = z.max(axis=1, keepdims=True)
    return z - m - np.log(np.exp(z - m).sum(axis=1, keepdims=True))


def torch_lerp(a, b, w):
    """ATen lerp: a + w*(b-a) if w < 0.5 else b - (b-a)*(1-w), float32."""
    a, b, w = F32(a), F32(b), F32(w)
    if w < F32(0.5):
        return F32(a + F32(w * F32(b - a)))
    return F32(b - F32(F32(b - a) * F32(F32(1.0) - w)))


def quantile_linear(values, q):
    """torch.quantile(v, q, interpolation='linear') restated in float32 (I/utils.py:481)."""
    v = np.sort(np.asarray(values, F32))
    qf = F32(q)
    rank = F32(qf * F32(len(v) - 1))
    lo = int(rank)
    hi = int(math.ceil(float(rank)))
    w = F32(rank - F32(lo))
    return torch_lerp(v[lo], v[hi], w)


def certainty_scores(q, use_entropy):
    """`DACPManager.calculate_certainty_scores` (I/utils.py:400-428); float32 like torch."""
    q = np.asarray(q, F32)
    pred = q.argmax(axis=1)
    mx = q.max(axis=1)
    if not use_entropy:
        return mx.astype(F32), pred
    ent = -np.sum(q * np.log2(q + F32(1e-8)), axis=1, dtype=F32)
    norm = (ent / F32(np.log2(q.shape[1]))).astype(F32)
    return (mx * (F32(1.0) - norm)).astype(F32), pred


# ------------------------------------------------------------------------ encoder

def encoder_forward(x, pad, W1, b1):
    """`Emotion2VecEncoder.forward` (I/model.py:18-41).

    x f32 [B,T,D], pad bool [B,T] (True = pad).  Returns (e [B,H], act_mask [B,T,H] bool,
    valid_len [B]) where act_mask = (pre > 0) & ~pad is what the weight gradient needs.
    """
    B, T, D = x.shape
    pre = (x.reshape(B * T, D) @ W1.T).reshape(B, T, -1) + b1
    valid = ~pad
    act = (pre > 0) & valid[..., None]
    summed = np.where(act, pre, F32(0)).sum(axis=1, dtype=F32)
    vlen = valid.sum(axis=1).astype(F32)
    e = (summed / np.maximum(vlen, F32(1.0))[:, None]).astype(F32)
    return e, act, vlen


def encoder_wgrad(x, act, vlen, de):
    """d/dW1, d/db1 of sum_b de_b . e_b through the masked mean pool + ReLU (I/model.py:28-36)."""
    B, T, D = x.shape
    scale = (np.asarray(de, np.float64) / np.maximum(vlen, 1.0)[:, None]).astype(F32)   # [B,H]
    G = np.where(act, scale[:, None, :], F32(0)).reshape(B * T, -1)                     # [BT,H]
    dW1 = G.T @ x.reshape(B * T, D)
    db1 = G.sum(axis=0, dtype=np.float64).astype(F32)
    return dW1.astype(F32), db1


# ---------------------------------------------------------------------- augmentation

def weak_augment(x, nw, std):
    """`weak_augment` (I/utils.py:328-331): x + randn*std."""
    return (x + (nw * F32(std)).astype(F32)).astype(F32)


def strong_augment(x, ns, u, start, std, p_feat, mask_ratio):
    """`strong_augment` + `_apply_temporal_masking` (I/utils.py:333-375).

    Noise, then ONE [D] feature mask shared by the batch (no rescale), then per-sample
    zeroing of int(Tmax*ratio) frames starting at start[b] (padded Tmax, I/utils.py:365-372).
    """
    out = (x + (ns * F32(std)).astype(F32)).astype(F32)
    if p_feat > 0:
        out = out * (u > F32(p_feat)).astype(F32)[None, None, :]
    B, T, _ = x.shape
    mlen = int(T * mask_ratio)
    if mask_ratio > 0 and mlen > 0:
        for b in range(B):
            s = int(start[b])
            out[b, s:s + mlen] = 0
    return out.astype(F32)


# ---------------------------------------------------------------------------- DACP

class DACPState:
    """`DACPManager` state (I/utils.py:384-398): Q (quality), tau (EMA thresholds), score sums."""

    def __init__(self, C, tau0=None, Q0=None):
        self.Q = np.full(C, 0.5, F32) if Q0 is None else np.asarray(Q0, F32).copy()
        self.tau = np.full(C, 0.5, F32) if tau0 is None else np.asarray(tau0, F32).copy()
        self.score_sum = np.zeros(C, np.float64)
        self.score_cnt = np.zeros(C, np.int64)

    def epoch_end(self, beta):
        """`update_class_quality_scores_epoch` (I/utils.py:430-447)."""
        cur = np.where(self.score_cnt > 0, self.score_sum / np.maximum(self.score_cnt, 1), self.Q)
        self.Q = (F32(beta) * self.Q + F32(1 - beta) * cur.astype(F32)).astype(F32)
        self.score_sum[:] = 0
        self.score_cnt[:] = 0


def dacp_mask(state, q, epoch, anchors, cfg, use_entropy):
    """`DACPManager.calculate_mask` (I/utils.py:449-507). Mutates state; returns (mask, s, pred, w)."""
    C = len(state.Q)
    s, pred = certainty_scores(q, use_entropy)
    delta = (state.Q - state.Q.mean(dtype=F32)).astype(F32)
    w = (F32(1.0) / (F32(1.0) + np.exp(-(F32(cfg["DACP_SENSITIVITY_K"]) * delta)))).astype(F32)
    gamma = cfg["DACP_QUANTILE_START"] + (cfg["DACP_QUANTILE_END"] - cfg["DACP_QUANTILE_START"]) * (
        epoch / cfg["EPOCHS"])
    that = np.zeros(C, F32)
    for c in range(C):
        sc = s[pred == c]
        that[c] = quantile_linear(sc, gamma) if len(sc) > 0 else state.tau[c]
    adj = (F32(cfg["DACP_CALIBRATION_STRENGTH_LAMBDA"]) * (w - F32(0.5))).astype(F32)
    floored = np.maximum((that + adj).astype(F32), np.asarray(anchors, F32))
    a = cfg["DACP_THRESHOLD_SMOOTHING_ALPHA"]
    state.tau = (F32(a) * state.tau + F32(1 - a) * floored).astype(F32)
    mask = s >= state.tau[pred]
    for c in range(C):
        sel = pred == c
        state.score_sum[c] += float(np.sum(s[sel], dtype=np.float64))
        state.score_cnt[c] += int(sel.sum())
    return mask, s, pred, w, floored


# ---------------------------------------------------------------------------- ECDA

def _gaussian_kernel_terms(Zs, Zt, ws, wt):
    """`ECDALoss._gaussian_kernel` (I/utils.py:521-563) + its analytic backward.

    Returns (mmd, dZs, dZt) for mmd = t_ss + t_tt - 2 t_st; the bandwidth is detached
    (`L2_dist.data`, I/utils.py:540) and weights carry no gradient.
    """
    ns, nt = len(Zs), len(Zt)
    Z = np.concatenate([Zs, Zt], 0).astype(np.float64)
    n = ns + nt
    diff = Z[:, None, :] - Z[None, :, :]
    Dm = (diff ** 2).sum(-1)
    bw = Dm.sum() / (n * n - n) if n > 1 else 1.0
    bw /= 2.0 ** (5 // 2)
    bws = [bw * 2.0 ** i for i in range(5)]
    K = sum(np.exp(-Dm / (b + 1e-8)) for b in bws)
    dKdD = sum(-np.exp(-Dm / (b + 1e-8)) / (b + 1e-8) for b in bws)
    ws = np.asarray(ws, np.float64)
    wt = np.asarray(wt, np.float64)
    Wss = np.outer(ws, ws).sum() + 1e-8
    Wtt = np.outer(wt, wt).sum() + 1e-8
    Wst = np.outer(ws, wt).sum() + 1e-8
    tss = (K[:ns, :ns] * np.outer(ws, ws)).sum() / Wss
    ttt = (K[ns:, ns:] * np.outer(wt, wt)).sum() / Wtt
    tst = (K[:ns, ns:] * np.outer(ws, wt)).sum() / Wst
    mmd = tss + ttt - 2 * tst
    dK = np.zeros((n, n))
    dK[:ns, :ns] = np.outer(ws, ws) / Wss
    dK[ns:, ns:] = np.outer(wt, wt) / Wtt
    dK[:ns, ns:] = -2 * np.outer(ws, wt) / Wst
    Cm = dK * dKdD
    Csym = Cm + Cm.T
    dZ = 2 * (Csym.sum(1)[:, None] * Z - Csym @ Z)
    return mmd, dZ[:ns], dZ[ns:]


def ecda_loss(ec, es, yc, pred, mask, scores, w, cfg, class_aware, fixed_thr_mode):
    """`ECDALoss.forward` (I/utils.py:565-652) with analytic grads w.r.t. ec, es.

    `w` is DACP's class weight [C], or ones(B) in fixed-threshold mode (I/train.py:420),
    in which case the class loop runs over range(B) (output-equivalent quirk).
    """
    ec = np.asarray(ec, np.float64)
    es = np.asarray(es, np.float64)
    gec = np.zeros_like(ec)
    ges = np.zeros_like(es)
    m = np.asarray(mask)
    if m.dtype != bool:                                  # I/utils.py:573-576
        m = m > cfg["FIXED_CONFIDENCE_THRESHOLD"]
    ncls = len(w)
    total = 0.0
    if class_aware:
        cents, members = {}, {}
        for c in range(ncls):
            sel = np.nonzero((pred == c) & m)[0]
            if len(sel) > 0:
                cents[c] = es[sel].mean(0)
                members[c] = sel
        vcls = sorted(cents)
        rep = 0.0
        drep = {}
        if len(vcls) > 1:
            npairs = len(vcls) * (len(vcls) - 1) // 2
            dsum = 0.0
            for a_i, a in enumerate(vcls):
                drep[a] = np.zeros(es.shape[1])
            for a_i, a in enumerate(vcls):
                for b in vcls[a_i + 1:]:
                    dv = cents[a] - cents[b]
                    nrm = np.sqrt((dv ** 2).sum())
                    dsum += nrm
                    g = dv / nrm if nrm > 0 else np.zeros_like(dv)
                    drep[a] += -g / npairs
                    drep[b] += g / npairs
            rep = -dsum / npairs
        wf = np.asarray(w, np.float64)
        att = np.exp(cfg["ECDA_CLASS_ATTENTION_LAMBDA"] * (wf.mean() - wf))
        gam, dlt = cfg["ECDA_COMPACTNESS_WEIGHT_GAMMA"], cfg["ECDA_REPULSION_WEIGHT_DELTA"]
        rep_coef = 0.0
        for c in range(ncls):
            si = np.nonzero(yc == c)[0]
            ti = np.nonzero((pred == c) & m)[0]
            if len(si) < 2 or len(ti) < 2:               # I/utils.py:609-610
                continue
            mmd, dzs, dzt = _gaussian_kernel_terms(ec[si], es[ti], np.ones(len(si)), scores[ti])
            cen = es[ti].mean(0)
            comp = ((es[ti] - cen) ** 2).sum(1).mean()
            total += att[c] * (mmd + gam * comp + dlt * rep)
            gec[si] += att[c] * dzs
            ges[ti] += att[c] * (dzt + gam * 2.0 / len(ti) * (es[ti] - cen))
            rep_coef += att[c] * dlt
        if rep_coef != 0.0 and len(vcls) > 1:
            for c in vcls:
                ges[members[c]] += rep_coef * drep[c] / len(members[c])
    else:
        ti = np.nonzero(m)[0]
        if len(ec) >= 2 and len(ti) >= 2:                # I/utils.py:633-650
            mmd, dzs, dzt = _gaussian_kernel_terms(ec, es[ti], np.ones(len(ec)), np.ones(len(ti)))
            total = mmd
            gec += dzs
            ges[ti] += dzt
    return total, gec, ges


# ------------------------------------------------------------------------ full step

class DADOracle:
    """Student/teacher parameters + Adam + DACP state, stepping like `train_epoch`'s body.

    `step()` restates `train_step` (I/train.py:397-471) followed by backward, clip,
    Adam and EMA (I/train.py:484-492); CASIA/EMODB variants per `cfg['flavor']`.
    """

    def __init__(self, W1, b1, W2, b2, cfg, anchors=None, tau0=None, Q0=None):
        self.cfg = cfg
        self.s = [np.array(W1, F32), np.array(b1, F32), np.array(W2, F32), np.array(b2, F32)]
        self.t = [p.copy() for p in self.s]                 # _init_teacher_network (I/model.py:200-209)
        self.m = [np.zeros_like(p) for p in self.s]
        self.v = [np.zeros_like(p) for p in self.s]
        self.nstep = 0
        C = cfg["NUM_CLASSES"]
        self.anchors = np.zeros(C, F32) if anchors is None else np.asarray(anchors, F32)
        self.dacp = DACPState(C, tau0, Q0)

    def load_state(self, st):
        """Overwrite params, Adam moments/step and DACP tau/Q (score accumulators are kept)."""
        self.s = [np.array(a, F32) for a in st["student"]]
        self.t = [np.array(a, F32) for a in st["teacher"]]
        self.m = [np.array(a, F32) for a in st["exp_avg"]]
        self.v = [np.array(a, F32) for a in st["exp_avg_sq"]]
        self.nstep = int(st["nstep"])
        self.dacp.tau = np.array(st["tau"], F32)
        self.dacp.Q = np.array(st["Q"], F32)

    # classifier with an explicit dropout keep-mask (nn.Dropout: input * keep/(1-p))
    @staticmethod
    def _cls(e, W2, b2, keep, p):
        if keep is None or p == 0:
            d = e
        else:
            d = (e * (keep.astype(F32) / F32(1 - p)).astype(F32)).astype(F32)
        return (d @ W2.T + b2).astype(F32), d

    def step(self, inp, epoch, lr=None, rng=None, allreduce=None, world=1):
        """One step on inputs ``inp`` (oracle/synth.make_step_inputs layout).

        If the injected draws are absent, they are sampled from ``rng`` (numpy Generator):
        that is the CPU-baseline mode, timing the same work the reference's step does.

        Data parallel (the build's DP contract): ``allreduce(vec)`` returns
        the SUM over ``world`` ranks of a float64 vector [grads | floored tau' | score-sum
        deltas | count deltas | losses].  Each rank's mask/losses are the reference on its own
        shard; the update uses the rank-mean gradient, the committed thresholds are
        alpha*tau + (1-alpha)*mean(tau'), and the epoch score statistics are summed.
        """
        cfg = self.cfg
        use_dacp, use_ecda, use_entropy, class_aware = effective_switches(cfg)
        w_kl, w_ecda, warm = loss_weights(cfg, epoch)
        if lr is None:
            lr = cosine_lr(cfg, epoch)
        p = cfg["DROPOUT_RATE"]
        W1, b1, W2, b2 = self.s
        xc, mc, yc = inp["xc"], inp["mc"], inp["yc"]
        B = xc.shape[0]
        C = W2.shape[0]
        out = {"epoch": epoch, "lr": lr, "w_kl": w_kl, "w_ecda": w_ecda}
        if "keep1" not in inp:
            inp = dict(inp)
            H = W1.shape[0]
            inp["keep1"] = rng.random((B, H), dtype=np.float32) >= p
            inp["keep2"] = rng.random((inp["xn"].shape[0], H), dtype=np.float32) >= p

        # ---- clean supervised branch (I/train.py:398-403)
        ec, act_c, vlen_c = encoder_forward(xc, mc, W1, b1)
        zc, dc = self._cls(ec, W2, b2, inp["keep1"], p)
        pc = softmax(zc)
        eps = cfg["LABEL_SMOOTHING_FACTOR"] if cfg["USE_LABEL_SMOOTHING"] else 0.0
        lsm = log_softmax(zc)
        ce = float(np.mean(-(1 - eps) * lsm[np.arange(B), yc] - eps / C * lsm.sum(1)))
        gzc = (pc - (1 - eps) * np.eye(C)[yc] - eps / C) / B
        out.update(e_clean=ec, z_clean=zc, supervised_ce_loss=ce)
        kl = 0.0
        ecda = 0.0
        gec = np.zeros_like(ec, dtype=np.float64)
        gW2 = np.zeros((C, W1.shape[0]))
        gb2 = np.zeros(C)
        gW1 = np.zeros_like(W1)
        gb1 = np.zeros_like(b1)
        if not warm:
            # ---- noisy distillation branch (I/train.py:405-460)
            xn, mn = inp["xn"], inp["mn"]
            if "nw" not in inp:
                inp = dict(inp)
                Bn, T, D = xn.shape
                inp["nw"] = rng.standard_normal(xn.shape, dtype=np.float32)
                inp["ns"] = rng.standard_normal(xn.shape, dtype=np.float32)
                inp["u"] = rng.random(D, dtype=np.float32)
                mlen = int(T * cfg["TEMPORAL_MASK_RATIO"])
                inp["start"] = rng.integers(0, max(1, T - mlen + 1), size=Bn)
            xw = weak_augment(xn, inp["nw"], cfg["WEAK_NOISE_STD"])
            xs = strong_augment(xn, inp["ns"], inp["u"], inp["start"], cfg["STRONG_NOISE_STD"],
                                p, cfg["TEMPORAL_MASK_RATIO"])
            Wt1, bt1, Wt2, bt2 = self.t
            et, _, _ = encoder_forward(xw, mn, Wt1, bt1)
            zt = (et @ Wt2.T + bt2).astype(F32)
            q = softmax(zt).astype(F32)
            if use_dacp:
                tau_before = self.dacp.tau.copy()
                sums_before = (self.dacp.score_sum.copy(), self.dacp.score_cnt.copy())
                mask, s, pred, w, floored = dacp_mask(self.dacp, q, epoch, self.anchors, cfg, use_entropy)
                out.update(tau_before=tau_before, tau_after=self.dacp.tau.copy(), w=w, floored=floored)
                maskf = mask.astype(np.float64)
                ecda_mask = mask
            else:                                        # I/train.py:417-420
                s = q.max(1).astype(F32)
                pred = q.argmax(1)
                maskf = (s >= F32(cfg["FIXED_CONFIDENCE_THRESHOLD"])).astype(np.float64)
                w = np.ones(len(s), F32)          # torch.ones_like(mask): noisy batch size
                ecda_mask = maskf.astype(F32)
            es, act_s, vlen_s = encoder_forward(xs, mn, W1, b1)
            zs, ds = self._cls(es, W2, b2, inp["keep2"], p)
            out.update(e_teacher=et, z_teacher=zt, q=q, score=s, pred=pred, mask=maskf.astype(F32),
                       e_strong=es, z_strong=zs)
            ges = np.zeros_like(es, dtype=np.float64)
            gzs = np.zeros((xn.shape[0], C))
            msum = maskf.sum()
            if msum > 1:                                  # I/train.py:444
                qd = q.astype(np.float64)
                ls = log_softmax(zs)
                xlogy = np.where(qd > 0, qd * np.log(np.where(qd > 0, qd, 1.0)), 0.0)
                kl = float(((xlogy - qd * ls).sum(1) * maskf).sum() / (msum + 1e-8))
                gzs = maskf[:, None] * (softmax(zs) - qd) / (msum + 1e-8)
                if use_ecda and w_ecda > 0:
                    ecda, g1, g2 = ecda_loss(ec, es, yc, pred, ecda_mask, s.astype(np.float64), w,
                                             cfg, class_aware, not use_dacp)
                    gec += w_ecda * g1
                    ges += w_ecda * g2
            gzs = w_kl * gzs
            # classifier backward, strong pass
            gW2 += gzs.T @ ds
            gb2 += gzs.sum(0)
            ges += (gzs @ W2.astype(np.float64)) * (inp["keep2"] / (1 - p) if p > 0 else 1.0)
            out["e_strong_grad"] = ges
            gw, gb = encoder_wgrad(xs, act_s, vlen_s, ges)
            gW1 += gw
            gb1 += gb
        # classifier backward, clean pass
        gW2 += gzc.T @ dc
        gb2 += gzc.sum(0)
        gec += (gzc @ W2.astype(np.float64)) * (inp["keep1"] / (1 - p) if p > 0 else 1.0)
        out["e_clean_grad"] = gec
        gw, gb = encoder_wgrad(xc, act_c, vlen_c, gec)
        gW1 = (gW1 + gw).astype(F32)
        gb1 = (gb1 + gb).astype(F32)
        grads = [gW1, gb1, gW2.astype(F32), gb2.astype(F32)]
        total = ce + w_kl * kl + w_ecda * ecda
        out.update(consistency_loss=kl, ecda_loss=ecda, total_loss=total, grads=[g.copy() for g in grads])
        if allreduce is not None and world > 1:
            dacp_on = use_dacp and not warm
            Cn = len(self.dacp.tau)
            fl = np.asarray(out["floored"], np.float64) if dacp_on else np.zeros(Cn)
            dsum = (self.dacp.score_sum - sums_before[0]) if dacp_on else np.zeros(Cn)
            dcnt = (self.dacp.score_cnt - sums_before[1]).astype(np.float64) if dacp_on else np.zeros(Cn)
            vec = np.concatenate([g.astype(np.float64).reshape(-1) for g in grads] +
                                 [fl, dsum, dcnt, np.array([total, ce, kl, ecda], np.float64)])
            vec = np.asarray(allreduce(vec), np.float64)
            o, new = 0, []
            for g in grads:
                new.append((vec[o:o + g.size] / world).astype(F32).reshape(g.shape))
                o += g.size
            grads = new
            if dacp_on:
                a = cfg["DACP_THRESHOLD_SMOOTHING_ALPHA"]
                mean_fl = (vec[o:o + Cn] / world).astype(F32)
                self.dacp.tau = (F32(a) * tau_before + F32(1 - a) * mean_fl).astype(F32)
                self.dacp.score_sum = sums_before[0] + vec[o + Cn:o + 2 * Cn]
                self.dacp.score_cnt = sums_before[1] + np.rint(vec[o + 2 * Cn:o + 3 * Cn]).astype(np.int64)
                out["tau_committed"] = self.dacp.tau.copy()
            out["losses_mean"] = vec[o + 3 * Cn:o + 3 * Cn + 4] / world
            out["grads_mean"] = [g.copy() for g in grads]

        # ---- clip_grad_norm_ (I/train.py:487-488)
        norms = [np.sqrt(np.sum(g.astype(np.float64) ** 2)) for g in grads]
        tn = float(np.sqrt(np.sum(np.square(norms))))
        out["clip_norm"] = tn
        if cfg["GRADIENT_CLIPPING"]:
            coef = min(1.0, cfg["MAX_GRAD_NORM"] / (tn + 1e-6))
            grads = [(g * F32(coef)).astype(F32) for g in grads]
        out["grads_clipped"] = grads

        # ---- Adam, L2 weight decay added to the grad (I/train.py:362,489; torch single-tensor Adam)
        self.nstep += 1
        b1c, b2c, epsA, wd = 0.9, 0.999, 1e-8, cfg["WEIGHT_DECAY"]
        bc1 = 1 - b1c ** self.nstep
        bc2 = 1 - b2c ** self.nstep
        for i in range(4):
            g = (grads[i] + F32(wd) * self.s[i]).astype(F32)
            self.m[i] = (self.m[i] + F32(1 - b1c) * (g - self.m[i])).astype(F32)
            self.v[i] = (self.v[i] * F32(b2c) + F32(1 - b2c) * g * g).astype(F32)
            denom = (np.sqrt(self.v[i]) / F32(math.sqrt(bc2)) + F32(epsA)).astype(F32)
            self.s[i] = (self.s[i] - F32(lr / bc1) * (self.m[i] / denom)).astype(F32)

        # ---- teacher EMA, post-warm-up only (I/train.py:491-492, I/model.py:211-223)
        if not warm:
            mom = cfg["EMA_MOMENTUM"]
            self.t = [(t * F32(mom) + s * F32(1.0 - mom)).astype(F32) for t, s in zip(self.t, self.s)]
        out["student"] = [p.copy() for p in self.s]
        out["teacher"] = [p.copy() for p in self.t]
        return out
