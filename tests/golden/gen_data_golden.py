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
            import dataload_casia_noisy
            np.random.seed(seed)                # the train-index shuffle uses the global NumPy RNG
            ds = dataload_casia_noisy.load_casia_noisy_data(prefix, {"angry": 0, "happy": 1, "neutral": 2, "sad": 3})
            loaders = dataload_casia_noisy.create_casia_noisy_speaker_isolated_loaders(
                ds, fold, bs, ["angry", "happy", "neutral", "sad"])
            for k, (ln, ld) in enumerate(zip(("noisy_student", "noisy_teacher", "noisy_val", "noisy_test"), loaders)):
                _record(out, ln, ld, 300 + k)
    np.savez_compressed(out_path, **out)
    return {k: (list(v.shape) if hasattr(v, "shape") else None) for k, v in out.items()}


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--case":
        print(json.dumps(run_case(sys.argv[2], os.path.join(HERE, sys.argv[2] + ".npz"))))
        return
    for name in CASES:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--case", name], capture_output=True, text=True)
        if r.returncode:
            sys.stderr.write(r.stdout + r.stderr)
            raise SystemExit("%s failed" % name)
        print(name, "ok")


if __name__ == "__main__":
    main()
