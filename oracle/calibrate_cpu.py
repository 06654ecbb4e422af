#!/usr/bin/env python3
"""Calibrate bench.py's CPU baseline (oracle/torch_cpu.py) against the reference itself.

Runs in the build container only (the reference never travels to the GPU box): times the
reference's step -- Trainer.train_step + backward + clip_grad_norm_ + Adam + teacher EMA,
I/train.py:484-492, built with object.__new__ as tests/golden/gen_golden.py does -- and
TorchCPUStep on the same synthetic B=64, T=300 batches (IEMOCAP config, epoch 60, the
reference's own torch RNG), each in its own process, at 1 and all container threads.
Writes profiles/r02_cpu_calibration.json with ratio = port step time / reference step time.

    python oracle/calibrate_cpu.py [--threads 1,8] [--steps 8]
"""
import argparse
import json
import os
import platform
import statistics
import subprocess
import sys
import time
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference/IEMOCAP/DAD-train-IEMOCAP"
B, T, EPOCH = 64, 300, 60


def _inputs(k):
    sys.path.insert(0, REPO)
    from oracle import synth
    return synth.make_step_inputs(0, k, B, T, ragged=False)


def run_reference(steps):
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    sys.modules["seaborn"] = types.ModuleType("seaborn")
    import matplotlib
    matplotlib.use("Agg")
    import numpy as np
    import torch
    import torch.nn as nn
    import torch.optim as optim
    sys.path.insert(1, REPO)
    from oracle import synth
    cfg = __import__("config")
    model_mod, utils, train = __import__("model"), __import__("utils"), __import__("train")
    tr = object.__new__(train.IEMOCAPCrossDomainTrainer)
    tr.device = torch.device("cpu")
    tr.WARMUP_EPOCHS = cfg.WARMUP_EPOCHS
    tr.target_ecda_weight = cfg.WEIGHT_ECDA
    tr.weight_ecda = 0.0
    tr.initial_consistency_weight = cfg.INITIAL_CONSISTENCY_WEIGHT
    tr.final_consistency_weight = cfg.FINAL_CONSISTENCY_WEIGHT
    tr.current_consistency_weight = tr.initial_consistency_weight
    tr.num_classes = 4
    tr.tracked_sample_indices = None
    tr.bias_analysis_log = []
    tr.model = model_mod.SSRLModel(cfg)
    W1, b1, W2, b2, _ = synth.init_weights(0)
    with torch.no_grad():
        m = tr.model
        for p, a in zip([m.student_encoder.pre_net.weight, m.student_encoder.pre_net.bias,
                         m.student_classifier.fc_layer.weight, m.student_classifier.fc_layer.bias], (W1, b1, W2, b2)):
            p.copy_(torch.from_numpy(a))
    tr.model._init_teacher_network()
    tr.optimizer = optim.Adam(tr.model.parameters(), lr=cfg.LEARNING_RATE, weight_decay=cfg.WEIGHT_DECAY)
    tr.ce_criterion = nn.CrossEntropyLoss(label_smoothing=cfg.LABEL_SMOOTHING_FACTOR)
    tr.kl_criterion = nn.KLDivLoss(reduction="none")
    tr.dacp_manager = utils.DACPManager(4, cfg.EPOCHS, tr.device)
    tr.ecda_criterion = utils.ECDALoss()
    tr.calibrated_anchors = torch.zeros(4)
    tr.augmenter = utils.DataAugmentation()
    tr.update_loss_weights(EPOCH)
    times, masks = [], []
    for k in range(steps + 2):
        inp = _inputs(k)
        clean = {"net_input": {"feats": torch.from_numpy(inp["xc"]), "padding_mask": torch.from_numpy(inp["mc"])},
                 "labels": torch.from_numpy(inp["yc"])}
        noisy = {"net_input": {"feats": torch.from_numpy(inp["xn"]), "padding_mask": torch.from_numpy(inp["mn"])}}
        t0 = time.perf_counter()
        tr.model.train()
        tr.optimizer.zero_grad()
        losses = tr.train_step(clean, noisy, EPOCH)
        losses["total_loss"].backward()
        torch.nn.utils.clip_grad_norm_(tr.model.parameters(), cfg.MAX_GRAD_NORM)
        tr.optimizer.step()
        tr.model.update_teacher_ema()
        _ = {k_: v.item() for k_, v in losses.items()}      # the loop's .item() calls (I/train.py:494-495)
        times.append(time.perf_counter() - t0)
        masks.append(float(losses["ecda_loss"]))
    return times[2:], masks


def run_port(steps):
    import torch
    sys.path.insert(0, REPO)
    from oracle import dad_oracle, synth, torch_cpu
    cfg = dad_oracle.make_cfg("iemocap")
    W1, b1, W2, b2, _ = synth.init_weights(0)
    st = torch_cpu.TorchCPUStep(W1, b1, W2, b2, cfg)
    times, ecda = [], []
    for k in range(steps + 2):
        inp = _inputs(k)
        t0 = time.perf_counter()
        out = st.step(inp, EPOCH)
        times.append(time.perf_counter() - t0)
        ecda.append(out["ecda_loss"])
    return times[2:], ecda


def child(kind, threads, steps):
    import torch
    torch.set_num_threads(threads)
    times, ecda = (run_reference if kind == "reference" else run_port)(steps)
    print(json.dumps({"kind": kind, "threads": threads, "times": times, "ecda_nonzero": sum(e != 0 for e in ecda)}))


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="1,%d" % len(os.sched_getaffinity(0)))
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--child", nargs=2)
    a = ap.parse_args()
    if a.child:
        child(a.child[0], int(a.child[1]), a.steps)
        return
    res = {"workload": "IEMOCAP DAD step B=%d T=%d epoch %d (CE+KL+ECDA), torch CPU, own RNG" % (B, T, EPOCH),
           "cpu_model": cpu_model(), "host_cpus": len(os.sched_getaffinity(0)), "torch": None, "by_threads": {}}
    for n in [int(x) for x in a.threads.split(",")]:
        row = {}
        for kind in ("reference", "port"):
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", kind, str(n), "--steps", str(a.steps)],
                               stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                               env=dict(os.environ, PYTHONDONTWRITEBYTECODE="1", OMP_NUM_THREADS=str(n)))
            if r.returncode != 0:
                print(r.stderr[-3000:])
                sys.exit(1)
            d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
            row[kind] = {"median_s": statistics.median(d["times"]), "steps": len(d["times"]),
                         "steps_with_ecda": d["ecda_nonzero"]}
        row["ratio_port_over_reference"] = row["port"]["median_s"] / row["reference"]["median_s"]
        res["by_threads"][str(n)] = row
        print(n, json.dumps(row))
    import torch
    res["torch"] = torch.__version__
    out = os.path.join(REPO, "profiles", "r02_cpu_calibration.json")
    json.dump(res, open(out, "w"), indent=1)
    print("wrote", out)


if __name__ == "__main__":
    main()
