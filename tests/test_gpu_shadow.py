"""The BF16 step's W1 shadows (bf16 copies of the student/teacher W1 in the encoder's fragment
order) follow the parameters (step.py `_param_key` / `refresh_shadow`).

* In-place writes to a parameter (`p.copy_` under no_grad, load_state_dict) are seen by the
  next step by themselves.
* Writes through `p.data` (the reference's model.py:204-223 style) use a detached alias with a
  version counter of its own: `_param_key` does not change, so the documented contract is to
  call `refresh_shadow()` after them.  With it, the step equals a step object that was loaded
  with the same weights from the start, bit for bit.
"""
import numpy as np
import pytest
import torch

import gpu_harness as gh
from oracle import dad_oracle, synth
from test_gpu_parity import _problem

pytestmark = pytest.mark.gpu


def _new_w1(st, scale):
    w = np.asarray(st["student"][0], np.float32) * np.float32(scale)
    return torch.from_numpy(w).cuda()


def _run(step, inp):
    o = gh.run_step(step, inp, 60)
    return o, np.concatenate([g.reshape(-1) for g in o["grads"]])


def test_writes_through_data_need_refresh_and_inplace_writes_do_not():
    cfg = dad_oracle.make_cfg("iemocap")
    inp = _problem(B=16, T=64, seed=8, Bn=16, Tn=64)
    st = synth.make_state(8, 1)
    w_new = _new_w1(st, 0.5)

    # reference: a step whose model holds the new W1 from the start
    st2 = dict(st)
    st2["student"] = [w_new.cpu().numpy()] + list(st["student"][1:])
    ref = gh.make_step(cfg, precision="bf16")
    gh.load_state(ref, st2)
    o_ref, g_ref = _run(ref, inp)

    # write through .data: the key does not see it; refresh_shadow() restores parity
    step = gh.make_step(cfg, precision="bf16")
    gh.load_state(step, st)
    w1 = step.model.student_encoder.pre_net.weight
    key0 = step._param_key()
    w1.data.copy_(w_new)
    assert step._param_key() == key0   # the documented limitation
    step.refresh_shadow()
    o1, g1 = _run(step, inp)
    assert o1["total_loss"] == o_ref["total_loss"]
    np.testing.assert_array_equal(g1, g_ref)

    # in-place write to the parameter itself: seen without a refresh
    step2 = gh.make_step(cfg, precision="bf16")
    gh.load_state(step2, st)
    w1b = step2.model.student_encoder.pre_net.weight
    key0 = step2._param_key()
    with torch.no_grad():
        w1b.copy_(w_new)
    assert step2._param_key() != key0
    o2, g2 = _run(step2, inp)
    assert o2["total_loss"] == o_ref["total_loss"]
    np.testing.assert_array_equal(g2, g_ref)
