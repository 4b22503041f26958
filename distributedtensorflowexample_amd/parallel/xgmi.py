"""xGMI one-shot all-reduce communicator (small buckets; opt-in).

Wraps ``csrc/kernels/xgmi_allreduce.hip`` / ``xgmi_comm.cpp``: every rank
exports an uncached IPC slot, the handles are exchanged through the
torch.distributed TCP store, and each ``allreduce_sum_`` is ONE kernel that
publishes, flags and sums straight from peer memory over the direct xGMI
links (protocol: ``docs/COMM.md``).  Graph-capturable (epochs live on the
device).  Only f32, and only up to ``max_numel`` elements: it exists for the
latency-bound 318 KB gradient of the MNIST MLP; RCCL (``comm.NativeComm``)
remains the default and the path for large buckets.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops import hip


class XgmiComm:
    def __init__(self, rank, world_size, max_numel, device=None, store=None,
                 key="dtfx/xgmi/0", timeout_s=2.0, protocol=None):
        self.rank, self.world_size = int(rank), int(world_size)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None
                                   else torch.device(device).index)
        self.timeout_s = float(timeout_s)
        self.max_numel = int(max_numel)
        # "ll": 8-byte {value, epoch} words (no flag round trip; world <= 8); "flag": slots +
        # per-block epoch flags (any world <= 16)
        self.protocol = protocol or ("ll" if self.world_size <= 8 else "flag")
        self._h = hip().XgmiAllReduce(self.rank, self.world_size, self.device.index,
                                      self.max_numel, self.protocol)
        if store is None:
            store = dist.distributed_c10d._get_default_store()
        store.set("%s/%d" % (key, self.rank), self._h.handle())
        handles = [bytes(store.get("%s/%d" % (key, j))) for j in range(self.world_size)]
        self._h.open(handles)

    def allreduce_sum_(self, t):
        if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
            raise ValueError("XgmiComm: contiguous f32 GPU tensors only")
        if t.numel() > self.max_numel:
            raise ValueError("XgmiComm: %d elements > max_numel %d" % (t.numel(), self.max_numel))
        self._h.all_reduce(t.data_ptr(), t.numel(), torch.cuda.current_stream().cuda_stream,
                           self.timeout_s)
        return t

    def mlp_wgrad(self, p, lr, x, ws, stats=True):
        """MNIST-MLP weight-gradient launch with the gradient all-reduce fused into its
        epilogue (protocol "push"): ``p -= lr * sum over ranks of the gradient``; see
        ``ops.mlp_step.step_xgmi``."""
        from ..ops._ext import ptr

        self._h.mlp_wgrad(ptr(p), float(lr), ptr(x), ptr(ws.buf), ptr(ws.ctr),
                          ptr(ws.stats) if stats else 0, ws.stats_ring, ws.B,
                          torch.cuda.current_stream().cuda_stream, self.timeout_s)

    def mlp_head(self, p, labels, ws, dz1A):
        """Factor engine: MLP head launch that also all-gathers every rank's backprop factors
        dz1 into ``dz1A`` [world, 112, BP] (protocol "push"); see ``ops.mlp_step.step_factor``."""
        from ..ops._ext import ptr

        self._h.mlp_head(ptr(p), ptr(labels), ptr(ws.buf), ptr(dz1A), ws.B,
                         torch.cuda.current_stream().cuda_stream, self.timeout_s)

    def mlp_wgrad_factor(self, p, lr, x, xstride, dz1A, ws, stats=True):
        """Factor engine: global dW1 from the gathered factors and every rank's batch
        (``x`` = this rank's batch, rank q's at ``x + (q - rank) * xstride`` elements),
        small-parameter gradients exchanged, SGD applied in place."""
        from ..ops._ext import ptr

        self._h.mlp_wgrad_factor(ptr(p), float(lr), ptr(x), int(xstride), ptr(dz1A), ptr(ws.buf),
                                 ptr(ws.ctr), ptr(ws.stats) if stats else 0, ws.stats_ring, ws.B,
                                 torch.cuda.current_stream().cuda_stream, self.timeout_s)

    def broadcast_(self, t, root=0):
        """Broadcast as a sum with zeros off the root (small control-path use)."""
        if self.rank != root:
            t.zero_()
        return self.allreduce_sum_(t)

    def check(self):
        """Raise if any all-reduce timed out waiting for a peer (synchronizes the device)."""
        torch.cuda.synchronize(self.device)
        if self._h.error():
            raise RuntimeError("xGMI all-reduce timed out waiting for a peer")

    def destroy(self):
        self._h.close()
