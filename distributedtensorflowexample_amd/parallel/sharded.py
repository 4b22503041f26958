"""ZeRO-1 sharded optimizer: the GPU form of the reference's PS sharding.

The reference can spread its variables over several ps tasks
(``replica_device_setter(ps_tasks, ...)``, worker.py:24-25; ``cluster_spec``
hard-codes one ps at main.py:47): each ps task owns a subset of the
parameters, receives every worker's gradient for them and applies the update
(``ApplyGradientDescent`` colocated with the variable, worker.py:79).  SURVEY.md
§2.3 names the MI355X-native shape of that idea: every GPU is the "ps" of an
equal 1/N slice of the parameters.

    backward:  bucket complete -> reduce-scatter on the comm stream
               (each rank receives the summed gradient of ITS slice only)
    step:      owner applies the optimizer to its slice (slots are slice-sized:
               optimizer state costs 1/N of the replicated form)
               -> all-gather the updated slice back into every replica

Reduce-scatter + all-gather move the same bytes per link as one ring
all-reduce, so sync steps cost the same on xGMI while optimizer memory and
optimizer HBM traffic drop by N -- the trade that matters for Adam on large
models (12 B of f32 state per parameter) sized for 288 GB per GPU.

Usage::

    ddp = DistributedDataParallel(model, comm, shard=True)   # bucket layout padded
    opt = ShardedOptimizer(AdamOptimizer(1e-3), ddp)
    ddp.reset(); loss.backward(); opt.step()                 # step() joins backward comm

Replicas stay bit-identical: every parameter element is updated by exactly one
rank and then copied to all others.
"""
from __future__ import annotations

import torch


class ShardedOptimizer:
    """Wraps a ``pkg.optim`` optimizer (``GradientDescentOptimizer``,
    ``MomentumOptimizer``, ``AdamOptimizer``) so it updates only this rank's
    slice of every bucket of a ``DistributedDataParallel(..., shard=True)``."""

    def __init__(self, optimizer, ddp):
        if not getattr(ddp, "shard", False):
            raise ValueError("ShardedOptimizer needs DistributedDataParallel(..., shard=True)")
        self.opt, self.ddp = optimizer, ddp
        self.comm, self.world, self.rank = ddp.comm, ddp.world_size, ddp.comm.rank

    def param_shard(self, b):
        """View of this rank's slice of bucket ``b`` in the flat parameter buffer."""
        lo, hi, _ = self.ddp.buckets[b]
        n = (hi - lo) // self.world
        return self.ddp.flat[lo + self.rank * n:lo + (self.rank + 1) * n]

    def state_numel(self):
        """Elements of optimizer state held by this rank (all slots, all buckets)."""
        return sum(t.numel() for t in self.opt._slots.values())

    def step(self, global_step=None):
        ddp = self.ddp
        ddp.finish()  # launches stragglers, joins the reduce-scatters
        if hasattr(self.opt, "_t"):  # Adam: one bias-correction step per global step
            self.opt._t += 1
        cs = ddp.comm_stream
        with torch.no_grad():
            for b, (lo, hi, _) in enumerate(ddp.buckets):
                p = self.param_shard(b)
                self.opt._apply(p, ddp.grad_shards[b], ("zero1", b))
                if self.world == 1:
                    continue
                # all-gather on the comm stream so bucket b's copy overlaps bucket b+1's update
                if cs is not None:
                    cs.wait_stream(torch.cuda.current_stream(ddp.device))
                    with torch.cuda.stream(cs):
                        self.comm.all_gather(ddp.flat[lo:hi], p.clone())
                else:
                    self.comm.all_gather(ddp.flat[lo:hi], p.clone())
            if cs is not None:
                torch.cuda.current_stream(ddp.device).wait_stream(cs)
            if global_step is not None:
                global_step.add_(1)
        return global_step


__all__ = ["ShardedOptimizer"]
