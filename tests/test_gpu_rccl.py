"""The RCCL transport of the data-parallel step (csrc/rccl_dp.hip through the C ABI) on the
one-GPU box: a single-rank communicator is created from a fresh unique id, the step's
[grads | extras] buffer is SUM-all-reduced in place on the step's stream (the identity for
one rank, bit for bit), the rank probe (ncclCommCount + an all-reduced 1.0) reports one rank,
and the communicator is destroyed.  RCCL refuses two ranks on one GPU, so the multi-rank
exchange runs only in the driver's multi-GPU bench (whose line reports `comm.ranks_seen`);
the DP arithmetic is covered by test_gpu_dp.py over gloo."""
import ctypes

import pytest
import torch

import dadpkg

pytestmark = pytest.mark.gpu
PKG = dadpkg.pkg()


def test_single_rank_rccl_allreduce_is_identity():
    L = PKG.lib()
    n = L.dad_comm_unique_id_bytes()
    assert n > 0
    uid = (ctypes.c_uint8 * n)()
    assert L.dad_comm_get_unique_id(uid) == 0
    handle = ctypes.c_void_p()
    assert L.dad_comm_init(ctypes.byref(handle), 1, uid, 0) == 0
    comm = PKG.DPComm(0, 1, handle)
    model = PKG.SSRLModel().cuda()
    step = PKG.DADStep(model, flavor="iemocap", precision="bf16", rng="counter", seed=3)
    g = torch.Generator(device="cuda").manual_seed(5)
    step.grad.copy_(torch.randn(step.grad.shape, device="cuda", generator=g))
    before = step.grad.clone()
    st = step._state_struct(0)
    stream = torch.cuda.current_stream().cuda_stream
    assert L.dad_comm_allreduce_grad(handle, st, stream) == 0
    torch.cuda.synchronize()
    assert torch.equal(step.grad, before)
    assert comm.ranks_seen() == 1
    assert L.dad_comm_init(ctypes.byref(ctypes.c_void_p()), 0, uid, 0) == 1001     # argument check
    comm.close()
    assert comm._comm is None
