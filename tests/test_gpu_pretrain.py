"""Clean supervised pre-training step (pretrain.py) on the MI355X against the reference's
BaseModel + Adam + CrossEntropyLoss run for the same steps (golden
tests/golden/pretrain_iemocap.npz from tests/golden/gen_pretrain_golden.py).  FP32 mode,
tolerance 1e-4 relative (the north_star's bound)."""
import numpy as np
import pytest
import torch

import dadpkg
from oracle import synth
from test_data_cpu import _golden

pytestmark = pytest.mark.gpu
PKG = dadpkg.pkg()
TOL = 1e-4


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(1e-6, np.max(np.abs(b))))


def test_pretrain_steps_match_reference_basemodel():
    g = _golden("pretrain_iemocap")
    seed, B, T, steps = int(g["seed"]), int(g["B"]), int(g["T"]), int(g["steps"])
    pre = PKG.pretrain.PretrainStep(lr=float(g["lr"]), weight_decay=float(g["wd"]), precision="fp32")
    W1, b1, W2, b2 = synth.base_weights(seed)
    pre.load_base_state_dict({"pre_net.weight": torch.from_numpy(W1), "pre_net.bias": torch.from_numpy(b1),
                              "post_net.weight": torch.from_numpy(W2), "post_net.bias": torch.from_numpy(b2)})
    for k in range(steps):
        inp = synth.make_step_inputs(seed, k, B, T)
        batch = {"net_input": {"feats": torch.from_numpy(inp["xc"]), "padding_mask": torch.from_numpy(inp["mc"])},
                 "labels": torch.from_numpy(inp["yc"])}
        loss, z = pre.step(batch)
        assert abs(float(loss) - float(g["losses"][k])) <= TOL * max(1.0, abs(float(g["losses"][k]))), k
        assert _rel(z.cpu().numpy(), g["logits"][k]) < TOL, k
    sd = pre.base_state_dict()
    w1 = sd["pre_net.weight"].numpy().reshape(-1)
    assert _rel(w1[g["w1_index"]], g["W1_s"]) < TOL
    assert abs(w1.astype(np.float64).sum() - float(g["W1_sum"])) < 1e-3 * max(1.0, abs(float(g["W1_sum"])))
    for n, key in (("b1", "pre_net.bias"), ("W2", "post_net.weight"), ("b2", "post_net.bias")):
        assert _rel(sd[key].numpy().reshape(-1), g[n + "_s"]) < TOL, n


def test_pretrained_checkpoint_loads_into_the_dad_model(tmp_path):
    """The pre-trainer's checkpoint format feeds SSRLModel.load_complete_pretrained_weights."""
    pre = PKG.pretrain.PretrainStep(precision="bf16")
    path = str(tmp_path / "best_model_fold_1.ckpt")
    torch.save(pre.base_state_dict(), path)
    m = PKG.SSRLModel().cuda()
    m.load_complete_pretrained_weights(path)
    m._init_teacher_network()                  # the reference's SSRLModel.__init__ order (I/model.py:100-122)
    for a, b in ((m.student_encoder.pre_net.weight, pre.model.student_encoder.pre_net.weight),
                 (m.teacher_classifier.fc_layer.bias, pre.model.student_classifier.fc_layer.bias)):
        assert torch.equal(a.detach().cpu(), b.detach().cpu())
