"""The PyTorch-CPU step (oracle/torch_cpu.py, bench.py's CPU baseline) computes the reference's
step: replayed on the golden variants with the injected draws, its losses and logits match
the fixtures.  (The baseline is timed with torch's own generator; this pins what it computes.)"""
import numpy as np
import pytest
import torch

import goldens
from oracle import torch_cpu

CASES = ["iemocap_default", "iemocap_global_mmd", "iemocap_fixed_thr", "casia_ecda_snr0", "emodb_b8"]


@pytest.mark.parametrize("name", CASES)
def test_torch_cpu_step_matches_goldens(name):
    torch.set_num_threads(4)
    d, spec, cfg = goldens.load(name)
    W1, b1, W2, b2 = goldens.problem(spec)
    anchors = np.asarray(spec.get("anchors", [0.0] * 4), np.float32)
    for s, epoch in goldens.schedule(d):
        st = goldens.state(spec, s)
        inp = goldens.step_inputs(spec, s)
        stp = torch_cpu.TorchCPUStep(W1, b1, W2, b2, cfg, anchors=anchors)
        stp.load_state(st)
        out = stp.step(inp, epoch, lr=float(d["s%d_lr" % s]), draws=inp)
        for k in ("total_loss", "supervised_ce_loss", "consistency_loss", "ecda_loss"):
            want = float(d["s%d_%s" % (s, k)])
            assert abs(out[k] - want) <= 1e-4 * max(1.0, abs(want)), (name, s, k, out[k], want)
        np.testing.assert_allclose(out["z_clean"].detach().numpy(), d["s%d_z_clean" % s], rtol=0, atol=1e-4)
        if epoch >= 30:
            np.testing.assert_allclose(out["z_strong"].detach().numpy(), d["s%d_z_strong" % s], rtol=0, atol=1e-4)
        assert abs(out["clip_norm"] - float(d["s%d_clip_norm" % s])) <= 1e-4 * max(1.0, float(d["s%d_clip_norm" % s]))
        np.testing.assert_allclose(stp.student[3].detach().numpy(), d["s%d_sb2" % s], rtol=0, atol=1e-6)
