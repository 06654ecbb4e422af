#!/usr/bin/env python3
"""Generate golden vectors by running the REFERENCE DAD step (this container only).

Imports one DAD-train-* tree of /root/reference per subprocess (their `config`,
`utils`, `model` module names collide), builds the trainer with
``object.__new__`` (its __init__ needs the absent datasets), injects
the six per-step random draws (oracle/synth.py) and records what the reference
computes.  Only outputs and seeds are stored; inputs are regenerated bit-exactly
from ``numpy.random.RandomState`` by the tests.

The reference never travels to the GPU box: only the .npz files written here do.

Usage:  python tests/golden/gen_golden.py            # all variants
        python tests/golden/gen_golden.py --variant iemocap_default
"""
import argparse
import json
import os
import subprocess
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

TREES = {
    "IEMOCAP": ("IEMOCAP/DAD-train-IEMOCAP", "config", "train", "IEMOCAPCrossDomainTrainer"),
    "CASIA": ("CASIA/DAD-train-CASIA", "config_casia", "train_CASIA", "FixedCASIACrossDomainTrainer"),
    "EMODB": ("EMODB/DAD-train-EMODB", "config_emodb", "train_emodb", "FixedEMODBCrossDomainTrainer"),
}

# Each step is an independent transition from a seeded state (oracle/synth.make_state):
# 2 warm-up, 2 ramp, 3 full-weight steps, then the epoch-end DACP quality update over the
# scores the post-warm-up steps collected.
SCHEDULE = [0, 0, 35, 35, 60, 60, 60, "epoch_end"]

VARIANTS = {
    "iemocap_default": dict(tree="IEMOCAP", B=16, T=20, seed=11, anchors=[0.02, 0.0, 0.0, 0.05]),
    "iemocap_global_mmd": dict(tree="IEMOCAP", B=16, T=20, seed=12, overrides=dict(
        USE_CLASS_AWARE_MMD=False, ECDA_COMPACTNESS_WEIGHT_GAMMA=0.0, ECDA_REPULSION_WEIGHT_DELTA=0.0)),
    "iemocap_no_entropy": dict(tree="IEMOCAP", B=16, T=20, seed=13, overrides=dict(USE_ENTROPY_IN_SCORE=False)),
    "iemocap_fixed_thr": dict(tree="IEMOCAP", B=16, T=20, seed=14, overrides=dict(USE_DACP=False)),
    "casia_default": dict(tree="CASIA", B=16, T=20, seed=21),
    "casia_fixed_ecda": dict(tree="CASIA", B=16, T=20, seed=22, overrides=dict(USE_ECDA=True)),
    "emodb_b8": dict(tree="EMODB", B=8, T=20, seed=31),
    "emodb_b16": dict(tree="EMODB", B=16, T=24, seed=32),
    "iemocap_t300": dict(tree="IEMOCAP", B=8, T=300, seed=41),
    "emodb_hi_tau": dict(tree="EMODB", B=8, T=20, seed=33, tau_range=[0.96, 0.995]),
    "iemocap_b64": dict(tree="IEMOCAP", B=64, T=40, seed=51),
    # the bench geometry (BASELINE configs[1]): one warm-up and two full-weight steps
    "iemocap_b64_t300": dict(tree="IEMOCAP", B=64, T=300, seed=61, schedule=[0, 60, 60, "epoch_end"]),
    # BASELINE configs[3]: CASIA with DACP + ECDA forced on (C/config_casia.py:85-86 overridden),
    # noisy branch at SNR 0 / 5 / 10 dB
    "casia_ecda_snr0": dict(tree="CASIA", B=16, T=40, seed=71, snr_db=0.0,
                            overrides=dict(USE_DACP=True, USE_ECDA=True)),
    "casia_ecda_snr5": dict(tree="CASIA", B=16, T=40, seed=73, snr_db=5.0,
                            overrides=dict(USE_DACP=True, USE_ECDA=True)),
    "casia_ecda_snr10": dict(tree="CASIA", B=16, T=40, seed=72, snr_db=10.0,
                             overrides=dict(USE_DACP=True, USE_ECDA=True)),
}

W1_SAMPLE = 1024          # sampled entries of the [256,768] tensors stored per step


def _w1_index():
    import numpy as np
    return np.random.RandomState(7).choice(256 * 768, W1_SAMPLE, replace=False)


def _summ(t, idx, prefix, out):
    """Store a big tensor as sampled entries + float64 checksums."""
    import numpy as np
    a = t.detach().cpu().numpy().astype(np.float32).reshape(-1)
    out[prefix + "_s"] = a[idx]
    a64 = a.astype(np.float64)
    out[prefix + "_sum"] = np.float64(a64.sum())
    out[prefix + "_sumsq"] = np.float64((a64 * a64).sum())


def run_variant(name, out_path):
    import numpy as np
    sys.dont_write_bytecode = True          # never write __pycache__ into /root/reference
    spec = VARIANTS[name]
    sub, cfg_name, train_name, cls_name = TREES[spec["tree"]]
    tree = os.path.join(REF, sub)
    sys.path.insert(0, tree)
    sys.path.insert(0, REPO)
    sys.modules["seaborn"] = types.ModuleType("seaborn")   # only used for heatmaps
    import matplotlib
    matplotlib.use("Agg")
    import torch
    import torch.nn as nn
    import torch.optim as optim
    torch.set_num_threads(4)
    from oracle import synth

    cfg = __import__(cfg_name)
    for k, v in spec.get("overrides", {}).items():
        setattr(cfg, k, v)
    model_mod = __import__("model")
    utils = __import__("utils")
    train = __import__(train_name)
    Trainer = getattr(train, cls_name)

    B, T, seed = spec["B"], spec["T"], spec["seed"]
    C = cfg.NUM_CLASSES
    W1, b1, W2, b2, _ = synth.init_weights(seed)

    tr = object.__new__(Trainer)
    tr.device = torch.device("cpu")
    tr.WARMUP_EPOCHS = cfg.WARMUP_EPOCHS
    tr.target_ecda_weight = cfg.WEIGHT_ECDA
    tr.weight_ecda = 0.0
    tr.weight_scl = 0.0
    tr.target_scl_weight = 0.0
    tr.initial_consistency_weight = cfg.INITIAL_CONSISTENCY_WEIGHT if cfg.PROGRESSIVE_TRAINING else cfg.WEIGHT_CONSISTENCY
    tr.final_consistency_weight = cfg.FINAL_CONSISTENCY_WEIGHT if cfg.PROGRESSIVE_TRAINING else cfg.WEIGHT_CONSISTENCY
    tr.current_consistency_weight = tr.initial_consistency_weight
    tr.num_classes = C
    tr.tracked_sample_indices = None
    tr.bias_analysis_log = []
    tr.model = model_mod.SSRLModel(cfg)
    with torch.no_grad():
        m = tr.model
        m.student_encoder.pre_net.weight.copy_(torch.from_numpy(W1))
        m.student_encoder.pre_net.bias.copy_(torch.from_numpy(b1))
        m.student_classifier.fc_layer.weight.copy_(torch.from_numpy(W2))
        m.student_classifier.fc_layer.bias.copy_(torch.from_numpy(b2))
    tr.model._init_teacher_network()
    tr.optimizer = optim.Adam(tr.model.parameters(), lr=cfg.LEARNING_RATE, weight_decay=cfg.WEIGHT_DECAY)
    tr.ce_criterion = nn.CrossEntropyLoss(label_smoothing=cfg.LABEL_SMOOTHING_FACTOR if cfg.USE_LABEL_SMOOTHING else 0.0)
    tr.kl_criterion = nn.KLDivLoss(reduction="none")
    tr.dacp_manager = utils.DACPManager(C, cfg.EPOCHS, tr.device)
    tr.ecda_criterion = utils.ECDALoss()
    anchors = np.asarray(spec.get("anchors", [0.0] * C), np.float32)
    tr.calibrated_anchors = torch.from_numpy(anchors.copy())
    tr.augmenter = utils.DataAugmentation()

    # ---- RNG injection -------------------------------------------------------
    queue = {"randn": [], "rand": [], "randint": [], "drop": []}
    real = (torch.randn_like, torch.rand, torch.randint)

    def fake_randn_like(x, *a, **k):
        v = queue["randn"].pop(0)
        assert tuple(v.shape) == tuple(x.shape)
        return v

    def fake_rand(*size, **k):
        v = queue["rand"].pop(0)
        return v

    def fake_randint(low, high, size, **k):
        v = queue["randint"].pop(0)
        assert 0 <= v < high, (v, high)
        return torch.tensor([v], dtype=torch.int64)

    class InjectedDropout(nn.Module):
        """nn.Dropout semantics (`noise.bernoulli_(1-p).div_(1-p)`; input*noise) with a given mask."""
        def __init__(self, p):
            super().__init__()
            self.p = p

        def forward(self, x):
            keep = queue["drop"].pop(0)
            noise = keep.to(torch.float32).div_(1 - self.p)
            return x * noise

    p = tr.model.student_classifier.dropout.p
    tr.model.student_classifier.dropout = InjectedDropout(p)

    # ---- capture hooks -----------------------------------------------------------
    cap = {}

    def hook(name):
        def f(mod, inp, out):
            cap.setdefault(name, []).append(out.detach().clone())
        return f

    tr.model.student_encoder.register_forward_hook(hook("s_enc"))
    tr.model.student_classifier.register_forward_hook(hook("s_cls"))
    tr.model.teacher_encoder.register_forward_hook(hook("t_enc"))
    tr.model.teacher_classifier.register_forward_hook(hook("t_cls"))
    real_cm = tr.dacp_manager.calculate_mask

    def wrapped_cm(probs, epoch, anchors_):
        cap["tau_before"] = tr.dacp_manager.ema_thresholds.detach().clone()
        cap["Q_before"] = tr.dacp_manager.class_quality_scores.detach().clone()
        mk, sc, w = real_cm(probs, epoch, anchors_)
        cap["dacp"] = (mk.detach().clone(), sc.detach().clone(), w.detach().clone())
        cap["tau_after"] = tr.dacp_manager.ema_thresholds.detach().clone()
        return mk, sc, w
    tr.dacp_manager.calculate_mask = wrapped_cm

    idx = _w1_index()
    out = {"w1_index": idx, "B": B, "T": T, "seed": seed, "anchors": anchors,
           "torch_version": torch.__version__}
    cfg_dump = {k: getattr(cfg, k) for k in dir(cfg) if k.isupper()
                and isinstance(getattr(cfg, k), (int, float, bool, str))}
    out["cfg_json"] = json.dumps(cfg_dump, default=str)
    out["variant_json"] = json.dumps(spec)

    student_params = [tr.model.student_encoder.pre_net.weight, tr.model.student_encoder.pre_net.bias,
                      tr.model.student_classifier.fc_layer.weight, tr.model.student_classifier.fc_layer.bias]
    teacher_params = [tr.model.teacher_encoder.pre_net.weight, tr.model.teacher_encoder.pre_net.bias,
                      tr.model.teacher_classifier.fc_layer.weight, tr.model.teacher_classifier.fc_layer.bias]

    step = 0
    torch.randn_like, torch.rand, torch.randint = fake_randn_like, fake_rand, fake_randint
    try:
        for item in spec.get("schedule", SCHEDULE):
            if item == "epoch_end":
                Q0 = synth.make_state(seed, step, C, tuple(spec.get("tau_range", (0.55, 0.9))))["Q"]
                tr.dacp_manager.class_quality_scores = torch.from_numpy(Q0.copy())
                out["epoch_end_counts"] = np.array([len(v) for v in tr.dacp_manager.batch_scores_per_class])
                tr.dacp_manager.update_class_quality_scores_epoch(tr.dacp_manager.batch_scores_per_class)
                out["epoch_end_after_step"] = step
                out["epoch_end_Q"] = tr.dacp_manager.class_quality_scores.numpy().copy()
                continue
            epoch = item
            pre = "s%d_" % step
            inp = synth.make_step_inputs(seed, step, B, T, snr_db=spec.get("snr_db", 5.0))
            st = synth.make_state(seed, step, C, tuple(spec.get("tau_range", (0.55, 0.9))))
            with torch.no_grad():
                for p_, a in zip(student_params, st["student"]):
                    p_.copy_(torch.from_numpy(a))
                for p_, a in zip(teacher_params, st["teacher"]):
                    p_.copy_(torch.from_numpy(a))
            for p_, ea, eas in zip(student_params, st["exp_avg"], st["exp_avg_sq"]):
                tr.optimizer.state[p_] = {"step": torch.tensor(float(st["nstep"])),
                                          "exp_avg": torch.from_numpy(ea.copy()),
                                          "exp_avg_sq": torch.from_numpy(eas.copy())}
            tr.dacp_manager.ema_thresholds = torch.from_numpy(st["tau"].copy())
            tr.dacp_manager.class_quality_scores = torch.from_numpy(st["Q"].copy())
            tr.update_loss_weights(epoch)
            lr = cfg.LEARNING_RATE * (1 + __import__("math").cos(__import__("math").pi * epoch / cfg.EPOCHS)) / 2
            for g in tr.optimizer.param_groups:
                g["lr"] = lr
            queue["drop"] = [torch.from_numpy(inp["keep1"]), torch.from_numpy(inp["keep2"])]
            queue["randn"] = [torch.from_numpy(inp["nw"]), torch.from_numpy(inp["ns"])]
            queue["rand"] = [torch.from_numpy(inp["u"])]
            queue["randint"] = [int(v) for v in inp["start"]]
            cap.clear()
            clean = {"net_input": {"feats": torch.from_numpy(inp["xc"]),
                                   "padding_mask": torch.from_numpy(inp["mc"])},
                     "labels": torch.from_numpy(inp["yc"])}
            noisy = {"net_input": {"feats": torch.from_numpy(inp["xn"]),
                                   "padding_mask": torch.from_numpy(inp["mn"])},
                     "labels": torch.from_numpy(inp["yn"])}
            tr.model.train()
            tr.optimizer.zero_grad()
            losses = tr.train_step(clean, noisy, epoch)
            losses["total_loss"].backward()
            norm = torch.nn.utils.clip_grad_norm_(tr.model.parameters(), cfg.MAX_GRAD_NORM)
            grads_clipped = [p_.grad.detach().clone() for p_ in student_params]
            tr.optimizer.step()
            warm = tr.is_warmup_phase(epoch)
            if not warm:
                tr.model.update_teacher_ema()
            warm_used = len(queue["drop"])
            out[pre + "epoch"] = epoch
            out[pre + "lr"] = lr
            out[pre + "w_kl"] = float(tr.current_consistency_weight)
            out[pre + "w_ecda"] = float(tr.weight_ecda)
            for k in ("total_loss", "supervised_ce_loss", "consistency_loss", "ecda_loss"):
                out[pre + k] = float(losses[k])
            out[pre + "e_clean"] = cap["s_enc"][0].numpy()
            out[pre + "z_clean"] = cap["s_cls"][0].numpy()
            if not warm:
                assert warm_used == 0 and not queue["randn"] and not queue["randint"]
                out[pre + "e_strong"] = cap["s_enc"][1].numpy()
                out[pre + "z_strong"] = cap["s_cls"][1].numpy()
                out[pre + "e_teacher"] = cap["t_enc"][0].numpy()
                out[pre + "z_teacher"] = cap["t_cls"][0].numpy()
                if "dacp" in cap:
                    mk, sc, w = cap["dacp"]
                    out[pre + "mask"] = mk.numpy().astype(np.float32)
                    out[pre + "score"] = sc.numpy()
                    out[pre + "w"] = w.numpy()
                    out[pre + "tau_before"] = cap["tau_before"].numpy()
                    out[pre + "tau_after"] = cap["tau_after"].numpy()
                    out[pre + "Q"] = cap["Q_before"].numpy()
                    pred = cap["t_cls"][0].argmax(1).numpy()
                    out[pre + "mask_margin"] = float(np.abs(sc.numpy() - cap["tau_after"].numpy()[pred]).min())
            out[pre + "clip_norm"] = float(norm)
            # pre-clip grads = clipped / coef (coef<=1); store both the norm and clipped grads
            out[pre + "exp_avg_b1"] = tr.optimizer.state[student_params[1]]["exp_avg"].numpy().copy()
            out[pre + "exp_avg_sq_W2"] = tr.optimizer.state[student_params[2]]["exp_avg_sq"].numpy().copy()
            _summ(grads_clipped[0], idx, pre + "gW1c", out)
            out[pre + "gb1c"] = grads_clipped[1].numpy()
            out[pre + "gW2c"] = grads_clipped[2].numpy()
            out[pre + "gb2c"] = grads_clipped[3].numpy()
            _summ(student_params[0], idx, pre + "sW1", out)
            out[pre + "sb1"] = student_params[1].detach().numpy().copy()
            out[pre + "sW2"] = student_params[2].detach().numpy().copy()
            out[pre + "sb2"] = student_params[3].detach().numpy().copy()
            _summ(teacher_params[0], idx, pre + "tW1", out)
            out[pre + "tb1"] = teacher_params[1].detach().numpy().copy()
            out[pre + "tW2"] = teacher_params[2].detach().numpy().copy()
            out[pre + "tb2"] = teacher_params[3].detach().numpy().copy()
            step += 1
    finally:
        torch.randn_like, torch.rand, torch.randint = real
    out["n_steps"] = step
    np.savez_compressed(out_path, **out)
    print("wrote", out_path, "steps", step)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if a.variant:
        run_variant(a.variant, a.out or os.path.join(HERE, a.variant + ".npz"))
        return
    for name in VARIANTS:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--variant", name],
                           cwd=HERE, env=dict(os.environ, PYTHONDONTWRITEBYTECODE="1"),
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        tail = r.stdout.strip().splitlines()[-1:] if r.stdout else []
        print(name, "rc", r.returncode, tail)
        if r.returncode != 0:
            print(r.stdout[-4000:])
            sys.exit(1)


if __name__ == "__main__":
    main()
