#!/usr/bin/env python3
"""Golden vectors for the clean pre-training step by running the REFERENCE BaseModel
(IEMOCAP/pretrain-and-processed-IEMOCAP/model.py) with the pre-trainer's optimizer and loss
(train_for_clean.py:154-155, 393-420: Adam(lr, weight_decay) on model.parameters(),
nn.CrossEntropyLoss()) for a few steps on seeded synthetic batches (oracle/synth), this
container only.  Stores per-step losses and logits and the final parameters (sampled entries +
float64 checksums); inputs are regenerated from the seeds by the tests.

Usage:  python tests/golden/gen_pretrain_golden.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/IEMOCAP/pretrain-and-processed-IEMOCAP"

SEED, B, T, STEPS, LR, WD = 61, 16, 24, 4, 2e-4, 1e-5


def main():
    import numpy as np
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    sys.path.insert(0, REPO)
    import torch
    from oracle import synth
    from model import BaseModel
    torch.set_num_threads(4)
    W1, b1, W2, b2 = synth.base_weights(SEED)
    m = BaseModel()
    with torch.no_grad():
        m.pre_net.weight.copy_(torch.from_numpy(W1))
        m.pre_net.bias.copy_(torch.from_numpy(b1))
        m.post_net.weight.copy_(torch.from_numpy(W2))
        m.post_net.bias.copy_(torch.from_numpy(b2))
    opt = torch.optim.Adam(m.parameters(), lr=LR, weight_decay=WD)
    crit = torch.nn.CrossEntropyLoss()
    m.train()
    out = {"seed": SEED, "B": B, "T": T, "steps": STEPS, "lr": LR, "wd": WD, "torch_version": torch.__version__}
    idx = np.random.RandomState(7).choice(256 * 768, 1024, replace=False)
    out["w1_index"] = idx
    losses, logits = [], []
    for k in range(STEPS):
        inp = synth.make_step_inputs(SEED, k, B, T)
        x, pm, y = torch.from_numpy(inp["xc"]), torch.from_numpy(inp["mc"]), torch.from_numpy(inp["yc"])
        opt.zero_grad()
        z = m(x, pm)
        loss = crit(z, y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
        logits.append(z.detach().numpy())
    out["losses"] = np.array(losses)
    out["logits"] = np.stack(logits)
    for n, p in (("W1", m.pre_net.weight), ("b1", m.pre_net.bias), ("W2", m.post_net.weight), ("b2", m.post_net.bias)):
        a = p.detach().numpy().reshape(-1)
        out[n + "_s"] = a[idx] if n == "W1" else a
        out[n + "_sum"] = np.float64(a.astype(np.float64).sum())
    np.savez_compressed(os.path.join(HERE, "pretrain_iemocap.npz"), **out)
    print("pretrain_iemocap ok", losses)


if __name__ == "__main__":
    main()
