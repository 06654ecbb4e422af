#!/usr/bin/env python3
"""Generate data-path golden vectors by running the REFERENCE loaders (this container only).

Writes seeded synthetic feature files in the reference's on-disk formats
(oracle/data_oracle.write_synthetic_split) to a temporary directory, runs the reference's
own loader functions on them (one subprocess per reference tree: their `config` /
`dataload_clean` module names collide), and records per loader and per batch what the
reference's DataLoader + collator produce: ids, padding masks, labels and float64 checksums
of the padded features.  The features themselves are regenerated from the seed by the
tests, so only outputs are stored.  The reference never travels to the GPU box: only the
.npz files written here do.

Loaders and RNG: before iterating each loader the generator calls torch.manual_seed(k)
(k = its position in the table), so the shuffled loaders' orders are pinned by the seed.

Eval path (eval_*.npz): the reference trainer's validate() and _run_anchor_calibration() on the
same kind of synthetic split, with seeded student/teacher weights (eval_weights): metrics,
confusion matrices, the teacher disagreement rate and the calibrated anchors.

Usage:  python tests/golden/gen_data_golden.py
"""
import json
import os
import subprocess
import sys
import tempfile
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

CASES = {
    # name: (tree, flavor, seed, n_utt, max_len, batch_size, fold)
    "data_iemocap": ("IEMOCAP/DAD-train-IEMOCAP", "iemocap", 5, 150, 40, 16, 2),
    "data_casia": ("CASIA/DAD-train-CASIA", "casia", 6, 90, 30, 8, 1),
    "data_emodb": ("EMODB/DAD-train-EMODB", "emodb", 8, 160, 30, 8, 4),
}


def _record(out, name, loader, seed):
    import numpy as np
    import torch
    torch.manual_seed(seed)
    ids, pads, labels, sums, sumsqs, shapes = [], [], [], [], [], []
    for batch in loader:
        x = batch["net_input"]["feats"].numpy().astype(np.float64)
        pads.append(batch["net_input"]["padding_mask"].numpy().reshape(-1))
        shapes.append(np.array(batch["net_input"]["feats"].shape[:2], np.int64))
        sums.append(x.sum())
        sumsqs.append((x * x).sum())
        if "id" in batch:
            ids.append(batch["id"].numpy())
        lab = batch.get("labels")
        labels.append(np.full(shapes[-1][0], -2, np.int64) if lab is None else lab.numpy().reshape(-1))
    out[name + "_shapes"] = np.stack(shapes)
    out[name + "_pad"] = np.concatenate(pads)
    out[name + "_labels"] = np.concatenate(labels)
    out[name + "_sum"] = np.array(sums)
    out[name + "_sumsq"] = np.array(sumsqs)
    if ids:
        out[name + "_ids"] = np.concatenate(ids)


def run_case(name, out_path):
    import numpy as np
    sys.dont_write_bytecode = True          # never write __pycache__ into /root/reference
    tree, flavor, seed, n_utt, max_len, bs, fold = CASES[name]
    sys.path.insert(0, os.path.join(REF, tree))
    sys.path.insert(0, REPO)
    sys.modules.setdefault("seaborn", types.ModuleType("seaborn"))
    import torch
    from oracle import data_oracle
    out = {"seed": np.int64(seed), "batch_size": np.int64(bs), "fold": np.int64(fold),
           "torch_version": np.array(torch.__version__)}
    with tempfile.TemporaryDirectory() as d:
        prefix = data_oracle.write_synthetic_split(d, seed, n_utt=n_utt, max_len=max_len, flavor=flavor)
        if flavor == "iemocap":
            import dataload_clean
            import dataload_noisy
            # raw parse with the length filter the pre-trainers use (min 3) and a max length
            _, sizes, offsets, labs = dataload_noisy.load_emotion2vec_dataset(prefix, min_length=3, max_length=30)
            out["parse_sizes"], out["parse_offsets"] = np.asarray(sizes), np.asarray(offsets)
            out["parse_labels"] = np.array(labs)
            out["session_ids"] = np.array(dataload_noisy.get_session_ids(prefix, n_utt))
            loaders = dataload_noisy.get_cv_dataloaders_noisy(d, bs, fold_id=fold)
            for k, (ln, ld) in enumerate(zip(("noisy_student", "noisy_teacher", "noisy_val", "noisy_test"), loaders)):
                _record(out, ln, ld, 100 + k)
            tr, va, te, _, _ = dataload_clean.get_cv_dataloaders(d, bs, fold_id=fold)
            for k, (ln, ld) in enumerate(zip(("clean_train", "clean_val", "clean_test"), (tr, va, te))):
                _record(out, ln, ld, 200 + k)
        else:
            mod = __import__("dataload_casia_noisy" if flavor == "casia" else "dataload_emodb_noisy")
            np.random.seed(seed)                # the train-index shuffle uses the global NumPy RNG
            load = mod.load_casia_noisy_data if flavor == "casia" else mod.load_emodb_noisy_data
            make = (mod.create_casia_noisy_speaker_isolated_loaders if flavor == "casia"
                    else mod.create_emodb_noisy_speaker_isolated_loaders)
            ds = load(prefix, {"angry": 0, "happy": 1, "neutral": 2, "sad": 3})
            loaders = make(ds, fold, bs, ["angry", "happy", "neutral", "sad"])
            for k, (ln, ld) in enumerate(zip(("noisy_student", "noisy_teacher", "noisy_val", "noisy_test"), loaders)):
                _record(out, ln, ld, 300 + k)
    np.savez_compressed(out_path, **out)
    return {k: (list(v.shape) if hasattr(v, "shape") else None) for k, v in out.items()}


EVAL_CASES = {
    # name: (seed, n_utt, max_len, batch_size, fold)
    "eval_iemocap": (7, 160, 40, 16, 3),
}


def run_eval_case(name, out_path):
    import numpy as np
    sys.dont_write_bytecode = True
    seed, n_utt, max_len, bs, fold = EVAL_CASES[name]
    sys.path.insert(0, os.path.join(REF, "IEMOCAP/DAD-train-IEMOCAP"))
    sys.path.insert(0, REPO)
    sys.modules.setdefault("seaborn", types.ModuleType("seaborn"))
    import matplotlib
    matplotlib.use("Agg")
    import collections
    import torch
    from oracle import data_oracle
    import config as cfg
    import dataload_clean
    import dataload_noisy
    import model as model_mod
    import train
    stu, tea = data_oracle.eval_weights(seed)
    tr = object.__new__(train.IEMOCAPCrossDomainTrainer)
    tr.device = torch.device("cpu")
    tr.WARMUP_EPOCHS = cfg.WARMUP_EPOCHS
    tr.current_epoch = 60
    tr.num_classes = 4
    tr.fold = fold - 1
    tr.class_names = list(cfg.LABEL_DICT)
    tr.training_history = collections.defaultdict(list)
    tr.model = model_mod.SSRLModel(cfg)
    with torch.no_grad():
        m = tr.model
        for net, (W1, b1, W2, b2) in (("student", stu), ("teacher", tea)):
            enc, cls = getattr(m, net + "_encoder"), getattr(m, net + "_classifier")
            enc.pre_net.weight.copy_(torch.from_numpy(W1))
            enc.pre_net.bias.copy_(torch.from_numpy(b1))
            cls.fc_layer.weight.copy_(torch.from_numpy(W2))
            cls.fc_layer.bias.copy_(torch.from_numpy(b2))
    out = {"seed": np.int64(seed), "batch_size": np.int64(bs), "fold": np.int64(fold),
           "torch_version": np.array(torch.__version__)}
    with tempfile.TemporaryDirectory() as d:
        data_oracle.write_synthetic_split(d, seed, n_utt=n_utt, max_len=max_len, flavor="iemocap")
        _, cval, ctest, _, _ = dataload_clean.get_cv_dataloaders(d, bs, fold_id=fold)
        _, _, nval, _ = dataload_noisy.get_cv_dataloaders_noisy(d, bs, fold_id=fold)
        for ln, ld, dom in (("clean_val", cval, "Clean"), ("clean_test", ctest, "Clean_Test"), ("noisy_val", nval, "Noisy")):
            r = tr.validate(ld, dom)
            for k in ("accuracy", "weighted_accuracy", "f1_weighted", "f1_macro"):
                out["%s_%s" % (ln, k)] = np.float64(r[k])
            for k in ("precision_per_class", "recall_per_class", "f1_per_class", "support_per_class"):
                out["%s_%s" % (ln, k)] = np.array(r[k])
            out[ln + "_confusion_matrix"] = np.asarray(r["confusion_matrix"])
        out["noisy_val_disagreement_rate"] = np.float64(tr.training_history["disagreement_rate_noisy"][-1])
        cfg.CLEAN_DATA_DIR, cfg.NOISY_DATA_DIR = d, d
        torch.manual_seed(seed)
        tr._run_anchor_calibration()
        out["calibrated_anchors"] = tr.calibrated_anchors.numpy().astype(np.float32)
        out["anchor_std_k"] = np.float64(cfg.ANCHOR_STD_K)
    np.savez_compressed(out_path, **out)
    return {k: (list(v.shape) if hasattr(v, "shape") else None) for k, v in out.items()}


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--case":
        fn = run_eval_case if sys.argv[2] in EVAL_CASES else run_case
        print(json.dumps(fn(sys.argv[2], os.path.join(HERE, sys.argv[2] + ".npz"))))
        return
    for name in list(CASES) + list(EVAL_CASES):
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--case", name], capture_output=True, text=True)
        if r.returncode:
            sys.stderr.write(r.stdout + r.stderr)
            raise SystemExit("%s failed" % name)
        print(name, "ok")


if __name__ == "__main__":
    main()
