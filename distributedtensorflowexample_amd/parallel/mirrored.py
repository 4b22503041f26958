"""Synchronous data parallelism (``MirroredStrategy``-style), MI355X-first.

Not in the reference (its only mode is async PS), but it is the north star of
BASELINE.json: every replica computes gradients on its own batch, gradients
are all-reduced over RCCL/xGMI and every replica applies the same averaged
update, so replicas stay bit-identical.

:class:`DistributedDataParallel` -- for arbitrary autograd models:

* parameters are re-homed into ONE flat buffer per dtype (views), gradients
  into a matching flat buffer, so optimizer kernels (ops/optim.py) and the
  all-reduce work on contiguous memory;
* the gradient buffer is cut into buckets (``bucket_mb``, default 32 MB -- big
  enough that each of the 7 xGMI links per MI355X carries a large chunk,
  small enough that the first bucket launches early in backward); buckets
  follow reverse parameter order (the order autograd produces gradients);
* a post-accumulate-grad hook per parameter counts arrivals; when a bucket
  is complete its all-reduce is launched on a dedicated comm stream that
  waits on the compute stream's event -- so communication overlaps the rest
  of backward; ``finish()`` joins the comm stream before the optimizer.

For the reference MLP itself, whose 318 KB gradient is produced by one fused
kernel, bucketing buys nothing; ``train/fused_mlp.FusedMLPTrainer`` takes the
all-reduce as a single graph-captured call instead.
"""
from __future__ import annotations

import torch


class DistributedDataParallel(torch.nn.Module):
    def __init__(self, module, comm, bucket_mb=32.0, broadcast_init=True, average=True,
                 shard=False):
        super().__init__()
        self.module = module
        self.comm = comm
        self.world_size = comm.world_size
        self.average = average
        params = [p for p in module.parameters() if p.requires_grad]
        if not params:
            raise ValueError("no trainable parameters")
        dev = params[0].device
        dtype = params[0].dtype
        if any(p.device != dev or p.dtype != dtype for p in params):
            raise ValueError("DDP flat buffers need a single device and dtype")
        self.device = dev
        n = sum(p.numel() for p in params)
        # buckets in reverse parameter order (gradient production order), each a contiguous
        # span of the flat buffer; 16-element alignment of every view keeps dwordx4 kernels
        # legal.  shard=True (ZeRO-1, parallel/sharded.py) pads every bucket to a multiple of
        # 16 * world so each rank owns an aligned 1/world slice of every bucket.
        self.shard = bool(shard)
        align = 16 * (self.world_size if self.shard else 1)
        sz = [(p.numel() + 15) // 16 * 16 for p in params]
        cap = max(1, int(bucket_mb * 2 ** 20 / params[0].element_size()))
        groups, cur, span = [], [], 0
        for i in reversed(range(len(params))):
            if cur and span + sz[i] > cap:
                groups.append(cur)
                cur, span = [], 0
            cur.append(i)
            span += sz[i]
        if cur:
            groups.append(cur)
        offs, off, spans = [0] * len(params), 0, {}
        for g in reversed(groups):  # ascending parameter order in memory
            lo = off
            for i in sorted(g):
                offs[i] = off
                off += sz[i]
            off = (off + align - 1) // align * align
            spans[id(g)] = (lo, off)
        self.flat = torch.zeros(off, device=dev, dtype=dtype)
        self.flat_grad = torch.zeros(off, device=dev, dtype=dtype)
        for p, o in zip(params, offs):
            self.flat[o:o + p.numel()].view_as(p).copy_(p.data)
            p.data = self.flat[o:o + p.numel()].view_as(p)
            p.grad = self.flat_grad[o:o + p.numel()].view_as(p)
        self.params, self.offsets, self.numel = params, offs, n
        self.buckets = [spans[id(g)] + (g,) for g in groups]  # (lo, hi, [param idx])
        # ZeRO-1: this rank's reduced gradient slice of every bucket (1/world of the buffer)
        self.grad_shards = ([torch.zeros((hi - lo) // self.world_size, device=dev, dtype=dtype)
                             for lo, hi, _ in self.buckets] if self.shard else None)
        self.bucket_of = {}
        for b, (_, _, idx) in enumerate(self.buckets):
            for i in idx:
                self.bucket_of[i] = b
        self._pending = [0] * len(self.buckets)
        self._launched = [False] * len(self.buckets)
        self.comm_stream = torch.cuda.Stream(dev) if dev.type == "cuda" else None
        self._hooks = []
        for i, p in enumerate(params):
            self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))
        if broadcast_init and self.world_size > 1:
            self.comm.broadcast_(self.flat, 0)
        self.reset()

    def _make_hook(self, i):
        def hook(p):
            b = self.bucket_of[i]
            self._pending[b] -= 1
            if self._pending[b] == 0:
                self._launch(b)
        return hook

    def _launch(self, b):
        lo, hi, _ = self.buckets[b]
        view = self.flat_grad[lo:hi]
        if self.comm_stream is not None:
            self.comm_stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.comm_stream):
                self._reduce(view, b)
        else:
            self._reduce(view, b)
        self._launched[b] = True

    def _reduce(self, view, b):
        if self.shard:  # reduce-scatter: this rank keeps only the slice it owns
            out = self.grad_shards[b]
            if self.world_size == 1:
                out.copy_(view)
                return
            self.comm.reduce_scatter(out, view)
            if self.average:
                out.div_(self.world_size)
            return
        if self.world_size == 1:
            return
        if self.average:
            if hasattr(self.comm, "allreduce_avg_"):
                self.comm.allreduce_avg_(view)
            else:
                self.comm.allreduce_sum_(view)
                view.div_(self.world_size)
        else:
            self.comm.allreduce_sum_(view)

    def reset(self):
        """Zero gradients and re-arm the bucket counters (call before backward)."""
        self.flat_grad.zero_()
        for b, (_, _, idx) in enumerate(self.buckets):
            self._pending[b] = len(idx)
            self._launched[b] = False

    zero_grad = reset

    def finish(self):
        """Launch any bucket whose hooks did not all fire; join the comm stream."""
        for b in range(len(self.buckets)):
            if not self._launched[b]:
                self._launch(b)
        if self.comm_stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.comm_stream)

    def forward(self, *a, **k):
        return self.module(*a, **k)


class MirroredStrategy:
    """Thin strategy object: comm + replica bookkeeping (tf.distribute-like)."""

    def __init__(self, comm):
        self.comm = comm
        self.num_replicas_in_sync = comm.world_size
        self.rank = comm.rank

    def wrap(self, module, **kw):
        return DistributedDataParallel(module, self.comm, **kw)

    def shard_optimizer(self, optimizer, ddp):
        """ZeRO-1: ``ddp = wrap(model, shard=True)``; the returned optimizer updates only
        this replica's slice of every bucket and all-gathers it (parallel/sharded.py)."""
        from .sharded import ShardedOptimizer

        return ShardedOptimizer(optimizer, ddp)

    def reduce_mean_(self, t):
        if self.num_replicas_in_sync > 1:
            self.comm.allreduce_sum_(t)
            t.div_(self.num_replicas_in_sync)
        return t

    def broadcast_(self, t, root=0):
        if self.num_replicas_in_sync > 1:
            self.comm.broadcast_(t, root)
        return t

    def check_replicas_identical(self, t):
        """Debug check: max over replicas of |t - t_rank0|."""
        return replica_divergence(self.comm, t, self.num_replicas_in_sync)


def replica_divergence(comm, t, world):
    """Max over replicas of |t - t_rank0| (0.0 when the sync replicas are bit-identical).
    Debug check of the deterministic sync mode: every step applies the same
    reduced gradient in the same order, so any nonzero value is a race or a lost update."""
    ref = t.detach().clone()
    if world > 1:
        comm.broadcast_(ref, 0)
    d = (t.detach() - ref).abs().max().reshape(1).float()
    if world > 1:
        comm.allreduce_max_(d)
    return float(d.item())


class ReplicaDivergenceError(RuntimeError):
    pass


def assert_replicas_identical(comm, t, world, step):
    d = replica_divergence(comm, t, world)
    if d != 0.0:
        raise ReplicaDivergenceError("replicas diverged at step %d: max |p - p_rank0| = %g"
                                     % (step, d))
