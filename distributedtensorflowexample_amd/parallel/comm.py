"""Collective communication for synchronous data parallelism.

The reference moves every gradient through a gRPC parameter server
(worker.py:75-85, 131-137).  The sync-DP replacement is a collective over
RCCL, one process per GPU, xGMI between the GPUs of a node:

* :class:`NativeComm` -- the framework's own RCCL communicator (C++,
  ``csrc/kernels/rccl_comm.cpp``).  Collectives are enqueued on the caller's
  current HIP stream, so a captured hipGraph replays them with no Python.
  The unique id travels through the torch.distributed TCP store; the process
  group itself may be gloo (control plane only).
* :class:`TorchComm` -- ``torch.distributed`` (``nccl`` backend = RCCL on
  ROCm, or ``gloo`` on CPU).  Used by the CPU test tier and as a fallback.

Both expose the same in-place API (``allreduce_sum_``, ``allreduce_avg_``,
``broadcast_``, ``reduce_scatter``, ``all_gather``, ``barrier``).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

_DT = {torch.float32: "float32", torch.float16: "float16", torch.bfloat16: "bfloat16",
       torch.float64: "float64", torch.int32: "int32", torch.int64: "int64",
       torch.uint8: "uint8"}


def _stream():
    return torch.cuda.current_stream().cuda_stream


class TorchComm:
    """torch.distributed-backed communicator (gloo on CPU, RCCL on GPU)."""

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)

    def allreduce_sum_(self, t):
        dist.all_reduce(t, group=self.group)
        return t

    def allreduce_avg_(self, t):
        dist.all_reduce(t, group=self.group)
        t.div_(self.world_size)
        return t

    def allreduce_max_(self, t):
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return t

    def broadcast_(self, t, root=0):
        dist.broadcast(t, root, group=self.group)
        return t

    def reduce_scatter(self, out, inp):
        if dist.get_backend(self.group) == "gloo":  # gloo has no reduce_scatter
            tmp = inp.clone()
            dist.all_reduce(tmp, group=self.group)
            n = out.numel()
            out.copy_(tmp.view(-1)[self.rank * n:(self.rank + 1) * n].view_as(out))
            return out
        dist.reduce_scatter_tensor(out, inp, group=self.group)
        return out

    def all_gather(self, out, inp):
        if dist.get_backend(self.group) == "gloo":
            parts = [torch.empty_like(inp) for _ in range(self.world_size)]
            dist.all_gather(parts, inp, group=self.group)
            out.copy_(torch.cat([p.view(-1) for p in parts]).view_as(out))
            return out
        dist.all_gather_into_tensor(out, inp, group=self.group)
        return out

    def all_to_all(self, out, inp):
        """Slice i (of world equal slices along dim 0) of ``inp`` goes to rank i; ``out``
        slice j comes from rank j."""
        dist.all_to_all_single(out, inp, group=self.group)
        return out

    def barrier(self):
        dist.barrier(group=self.group)


class NativeComm:
    """The framework's C++ RCCL communicator (GPU tensors only)."""

    def __init__(self, rank, world_size, device=None, store=None, key="dtfx/rccl/uid/0"):
        from ..ops import hip

        self._h = hip()
        self.rank, self.world_size = int(rank), int(world_size)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None
                                   else torch.device(device).index)
        if store is None:
            store = dist.distributed_c10d._get_default_store()
        if self.rank == 0:
            uid = self._h.rccl_unique_id()
            store.set(key, uid)
        else:
            uid = store.get(key)
        self._comm = self._h.RcclComm(bytes(uid), self.world_size, self.rank, self.device.index)

    @classmethod
    def from_process_group(cls, group=None, key="dtfx/rccl/uid/0"):
        return cls(dist.get_rank(group), dist.get_world_size(group), key=key)

    def _check(self, t):
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("NativeComm works on contiguous GPU tensors")
        return _DT[t.dtype]

    def allreduce_sum_(self, t):
        self._comm.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), self._check(t), "sum",
                              _stream())
        return t

    def allreduce_avg_(self, t):
        self._comm.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), self._check(t), "avg",
                              _stream())
        return t

    def allreduce_max_(self, t):
        self._comm.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), self._check(t), "max",
                              _stream())
        return t

    def broadcast_(self, t, root=0):
        self._comm.broadcast(t.data_ptr(), t.data_ptr(), t.numel(), self._check(t), int(root),
                             _stream())
        return t

    def reduce_scatter(self, out, inp):
        self._comm.reduce_scatter(inp.data_ptr(), out.data_ptr(), out.numel(), self._check(inp),
                                  "sum", _stream())
        return out

    def all_gather(self, out, inp):
        self._comm.all_gather(inp.data_ptr(), out.data_ptr(), inp.numel(), self._check(inp),
                              _stream())
        return out

    def all_to_all(self, out, inp):
        self._comm.all_to_all(inp.data_ptr(), out.data_ptr(), inp.numel() // self.world_size,
                              self._check(inp), inp.element_size(), _stream())
        return out

    def barrier(self):
        t = torch.zeros(1, device=self.device)
        self.allreduce_sum_(t)
        torch.cuda.current_stream().synchronize()

    def destroy(self):
        self._comm.destroy()

    def abort(self):
        """ncclCommAbort: unblock RCCL kernels waiting on a dead peer (watchdog teardown)."""
        self._comm.abort()

    def failed(self):
        """RCCL reported an asynchronous error (a remote failure or an abort)."""
        return self._comm.async_error() != 0


def make_comm(kind="auto", group=None):
    """``native`` (C++ RCCL), ``torch`` (torch.distributed) or ``auto``."""
    if kind == "auto":
        kind = "native" if torch.cuda.is_available() and os.environ.get(
            "DTFX_COMM", "native") == "native" else "torch"
    if kind == "native":
        return NativeComm.from_process_group(group)
    return TorchComm(group)


def make_comm_stream(device):
    """The stream the gradient-bucket all-reduces run on (overlapping the backward).
    ``DTFX_COMM_PRIORITY``: its HIP stream priority (torch's convention: lower = higher
    priority; ``torch.cuda.Stream.priority_range()``); unset: the default priority.  Measured
    on the simulated world-8 step (tools/probes/dp_sim.py)."""
    prio = os.environ.get("DTFX_COMM_PRIORITY")
    if prio is None or prio == "":
        return torch.cuda.Stream(device)
    return torch.cuda.Stream(device, priority=int(prio))
