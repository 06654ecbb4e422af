"""Seeded synthetic DAD problems (TEST INFRASTRUCTURE — checker side only).

Shared by the golden generator (tests/golden/gen_golden.py), the parity tests,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py``.
Nothing in the product package imports this module.

Every array comes from ``numpy.random.RandomState`` whose legacy stream is frozen
across NumPy versions, so a fixture only has to store its seed: the inputs are
regenerated bit-exactly on any host ("Golden vectors").

Shapes follow the reference collator (`I/dataload_noisy.py:111-129`):
feats f32 [B, Tmax, 768] zero-padded, padding_mask bool [B, Tmax] (True = pad),
labels int64 [B].  The six per-step random draws of the reference step, in the
order the reference consumes them ("Per-step RNG consumption"):

1. dropout keep-mask #1 [B, H]   (student classifier, clean pass, `I/train.py:400`)
2. N_w [B, T, D]                  (weak aug `torch.randn_like`, `I/utils.py:330`)
3. N_s [B, T, D]                  (strong aug `torch.randn_like`, `I/utils.py:338`)
4. u   [D]                        (feature dropout `torch.rand`, `I/utils.py:343`)
5. start [B]                      (temporal mask `torch.randint`, `I/utils.py:370`)
6. dropout keep-mask #2 [B, H]   (student classifier, strong pass, `I/train.py:440`)
"""
import numpy as np

D_IN = 768
H_DIM = 256
N_CLS = 4


def temporal_mask_len(tmax, ratio):
    """`int(seq_len * self.temporal_mask_ratio)` (I/utils.py:365), float64 like Python."""
    return int(tmax * ratio)


def init_weights(seed, D=D_IN, H=H_DIM, C=N_CLS, margin=5.0):
    """Student weights for a synthetic problem.

    W1/b1 follow nn.Linear's U(-1/sqrt(fan_in), 1/sqrt(fan_in)) range; W2 is set so
    the (teacher = student) classifier is confident on the class prototypes, which
    is what makes the DACP mask non-trivial and the ECDA gates pass.
    Returns (W1[H,D], b1[H], W2[C,H], b2[C], P[C,D]) float32.
    """
    rs = np.random.RandomState(seed)
    P = rs.normal(0.0, 2.0, size=(C, D))
    k1 = 1.0 / np.sqrt(D)
    W1 = rs.uniform(-k1, k1, size=(H, D))
    b1 = rs.uniform(-k1, k1, size=(H,))
    mu = np.maximum(P @ W1.T + b1, 0.0)             # embedding of each prototype
    dirs = mu - mu.mean(axis=0, keepdims=True)
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    proj = mu @ dirs.T                              # prototype logits per unit scale
    gap = np.mean([proj[c, c] - np.max(np.delete(proj[c], c)) for c in range(C)])
    W2 = (margin / gap) * dirs                      # ~`margin` logit gap on prototypes
    k2 = 1.0 / np.sqrt(H)
    b2 = rs.uniform(-k2, k2, size=(C,)) * 0.1
    f = np.float32
    return W1.astype(f), b1.astype(f), W2.astype(f), b2.astype(f), P.astype(f)


def make_batch(P, seed, B, T, snr_db=5.0, noisy=False, ragged=True, label_shift=0):
    """One collated batch: feats [B,T,D] f32, padding_mask [B,T] bool, labels [B] int64."""
    rs = np.random.RandomState(seed)
    C, D = P.shape
    labels = (np.arange(B) + label_shift) % C
    rs.shuffle(labels)
    if ragged:
        lengths = rs.randint(max(1, T // 2), T + 1, size=B)
        lengths[rs.randint(0, B)] = T          # the collator pads to the batch max
    else:
        lengths = np.full(B, T)
    sigma = 0.5 + (10.0 ** (-snr_db / 20.0) if noisy else 0.0)
    if noisy:   # per-utterance noise level spreads the teacher's certainty scores
        sigma = sigma * rs.uniform(0.5, 2.5, size=(B, 1, 1))
    x = P[labels][:, None, :] + sigma * rs.standard_normal(size=(B, T, D))
    pad = np.arange(T)[None, :] >= lengths[:, None]
    x[pad] = 0.0
    return x.astype(np.float32), pad, labels.astype(np.int64)


def make_draws(seed, B, T, D=D_IN, H=H_DIM, p_drop=0.1, mask_ratio=0.1):
    """The six injected random draws of one post-warm-up step (see module doc)."""
    rs = np.random.RandomState(seed)
    keep1 = rs.uniform(size=(B, H)) >= p_drop
    nw = rs.standard_normal(size=(B, T, D)).astype(np.float32)
    ns = rs.standard_normal(size=(B, T, D)).astype(np.float32)
    u = rs.uniform(size=(D,)).astype(np.float32)
    mlen = temporal_mask_len(T, mask_ratio)
    start = rs.randint(0, max(1, T - mlen + 1), size=B).astype(np.int64)
    keep2 = rs.uniform(size=(B, H)) >= p_drop
    return dict(keep1=keep1, nw=nw, ns=ns, u=u, start=start, keep2=keep2)


def make_step_inputs(problem_seed, step, B, T, snr_db=5.0, ragged=True):
    """Clean + noisy batches and the injected draws of step ``step``."""
    base = problem_seed * 7919 + step * 104729
    _, _, _, _, P = init_weights(problem_seed)
    xc, mc, yc = make_batch(P, base + 1, B, T, ragged=ragged, label_shift=0)
    xn, mn, yn = make_batch(P, base + 2, B, T, snr_db=snr_db, noisy=True,
                            ragged=ragged, label_shift=1)
    draws = make_draws(base + 3, B, T)
    return dict(xc=xc, mc=mc, yc=yc, xn=xn, mn=mn, yn=yn, **draws)


def make_state(problem_seed, step, C=N_CLS, tau_range=(0.55, 0.9)):
    """Seeded full training state at the START of golden step ``step``.

    Every golden step is an independent state transition (SURVEY §8(b) parity is per step
    "on identical inputs"): chained steps would diverge chaotically, because Adam's
    update m/sqrt(v) amplifies roundoff in tiny gradient entries to O(lr) parameter changes.
    Returns student/teacher params [W1,b1,W2,b2], Adam exp_avg/exp_avg_sq, Adam step count,
    DACP tau (EMA thresholds) and Q (class quality).
    """
    W1, b1, W2, b2, _ = init_weights(problem_seed)
    rs = np.random.RandomState(problem_seed * 31337 + step * 7)
    f = np.float32
    stud = [p + (0.004 * rs.standard_normal(p.shape)).astype(f) for p in (W1, b1, W2, b2)]
    teach = [p + (0.002 * rs.standard_normal(p.shape)).astype(f) for p in stud]
    m = [(0.003 * rs.standard_normal(p.shape)).astype(f) for p in stud]
    v = [((0.01 * rs.uniform(0.3, 1.5, size=p.shape)) ** 2).astype(f) for p in stud]
    nstep = 5 + 3 * step
    tau = rs.uniform(tau_range[0], tau_range[1], size=C).astype(f)
    Q = rs.uniform(0.3, 0.7, size=C).astype(f)
    return dict(student=[x.astype(f) for x in stud], teacher=[x.astype(f) for x in teach],
                exp_avg=m, exp_avg_sq=v, nstep=nstep, tau=tau, Q=Q)


def base_weights(seed):
    """BaseModel (IP/model.py:4-21) weights for the pre-training fixtures: init_weights(seed)
    with the classifier scaled back to nn.Linear's range (W2 / 40)."""
    W1, b1, W2, b2, _ = init_weights(seed)
    return W1, b1, (W2 / 40.0).astype(W2.dtype), b2
