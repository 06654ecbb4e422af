"""Data-parallel gradient exchange: one RCCL all-reduce per step over xGMI.

The reference is single-device (I/train.py:58).  Each rank runs the full DAD step on its
own clean+noisy shard; `dad_step_compute` leaves [grads | DACP tau', score sums, counts |
losses] in one flat buffer, this module SUM-all-reduces it in place on the step's stream
(RCCL, called through the C ABI so the collective is part of the enqueued step), and
`dad_step_apply` averages and applies it identically on every rank.
The RCCL communicator is bootstrapped by broadcasting rank 0's ncclUniqueId over the
already-initialised torch.distributed process group.
"""
import ctypes

import torch

from . import _lib


class DPComm:
    def __init__(self, rank, world, comm_handle=None):
        self.rank, self.world = int(rank), int(world)
        self._comm = comm_handle

    @classmethod
    def from_torch_distributed(cls, group=None):
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        if world == 1:
            return cls(rank, world, None)
        L = _lib.lib()
        n = L.dad_comm_unique_id_bytes()
        buf = (ctypes.c_uint8 * n)()
        if rank == 0:
            _lib.check(L.dad_comm_get_unique_id(buf), "dad_comm_get_unique_id")
        t = torch.tensor(list(bytes(buf)), dtype=torch.uint8)
        backend = dist.get_backend(group)
        if backend == "nccl":
            t = t.cuda()
        dist.broadcast(t, src=0, group=group)
        raw = bytes(t.cpu().tolist())
        idbuf = (ctypes.c_uint8 * n).from_buffer_copy(raw)
        handle = ctypes.c_void_p()
        _lib.check(L.dad_comm_init(ctypes.byref(handle), world, idbuf, rank), "dad_comm_init")
        return cls(rank, world, handle)

    def allreduce_grad(self, state_struct, stream, grad=None):
        if self.world == 1:
            return
        _lib.check(_lib.lib().dad_comm_allreduce_grad(self._comm, state_struct, stream), "dad_comm_allreduce_grad")

    def ranks_seen(self, device=None):
        """Ranks the RCCL transport actually connected: a float 1.0 per rank SUM-all-reduced
        through the communicator (checked against ncclCommCount)."""
        if self._comm is None:
            return 1
        L = _lib.lib()
        cnt = ctypes.c_int(0)
        _lib.check(L.dad_comm_count(self._comm, ctypes.byref(cnt)), "dad_comm_count")
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        one = torch.ones(1, device=dev)
        stream = torch.cuda.current_stream(dev)
        _lib.check(L.dad_comm_allreduce_f32(self._comm, one.data_ptr(), 1, stream.cuda_stream),
                   "dad_comm_allreduce_f32")
        seen = int(round(float(one.item())))
        if seen != cnt.value:
            raise _lib.DadError("RCCL all-reduce saw %d ranks, communicator has %d" % (seen, cnt.value))
        return seen

    def close(self):
        if self._comm is not None:
            _lib.lib().dad_comm_destroy(self._comm)
            self._comm = None


class ProcessGroupComm:
    """The same exchange over an existing torch.distributed process group (any backend).

    `DPComm` (RCCL through the C ABI) is the production path.  This one issues the SUM
    all-reduce of the step's [grads | tau' | score sums | counts | losses] buffer with
    torch.distributed on the current stream, so the data-parallel step can also run
    where RCCL cannot, e.g. several ranks sharing one GPU over gloo (tests, rehearsals).
    """

    def __init__(self, group=None):
        import torch.distributed as dist
        self._dist = dist
        self.group = group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)

    def allreduce_grad(self, state_struct, stream, grad=None):
        if self.world == 1:
            return
        if grad is None:
            raise ValueError("ProcessGroupComm needs the grad tensor")
        self._dist.all_reduce(grad, op=self._dist.ReduceOp.SUM, group=self.group)

    def ranks_seen(self, device=None):
        """Ranks the process group actually connected (a 1 per rank, SUM-all-reduced)."""
        one = torch.ones(1)
        self._dist.all_reduce(one, op=self._dist.ReduceOp.SUM, group=self.group)
        return int(round(float(one.item())))

    def close(self):
        pass
