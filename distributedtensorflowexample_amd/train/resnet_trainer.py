"""Data-parallel ResNet-50 trainer (north-star config 4 of BASELINE.json).

MirroredStrategy-style synchronous SGD: one process per GPU, per-block
gradient buckets all-reduced (sum) on a comm stream as soon as the block's
backward is done, then one fused momentum-SGD launch (f32 master, bf16 copy,
1/world folded in).  The step can be captured in a hipGraph.  The reference
has no counterpart (it trains an MLP with async PS, worker.py:71-79).

Owner-sharded optimizer (``zero1``; DTFX_RESNET_ZERO1=1 turns it on for world > 1): the
reference applies each gradient once, on the ps task that owns the variable
(``apply_gradients`` colocated with it, worker.py:75-79, placed by ``replica_device_setter``,
worker.py:24-25).  Every GPU owns an equal 1/W shard of each bucket (stem, bottleneck blocks,
head -- padded to ALIGN * W elements):

    backward      bucket i final -> reduce-scatter on the comm stream: this rank holds the
                  summed gradient of its shard
    after it      momentum SGD on the shard only (1/W of the optimizer's work)
    next step     all-gather of the shards (f32 master + bf16 working copy) on the comm
                  stream at the start of the step; the forward of block b waits only for
                  bucket b's gather (``on_bucket_needed``), so the gathers overlap the forward

Between steps the non-owned shards are one update behind: ``sync_params()`` (a collective)
completes them for checkpoints, evals and replica checks.
"""
from __future__ import annotations

import os

import torch

from ..models.resnet import STAGES, ResNet50, synthetic_imagenet


class ResNetTrainer:
    def __init__(self, batch, device, comm=None, lr=0.1, momentum=0.9, wd=5e-5, seed=0,
                 image_size=224, stages=STAGES, num_classes=1000, overlap=True, data_seed=0,
                 zero1=None):
        self.batch = batch
        self.device = torch.device(device)
        self.comm = comm
        self.world = comm.world_size if comm is not None else 1
        self.lr, self.momentum, self.wd = lr, momentum, wd
        if zero1 is None:
            zero1 = os.environ.get("DTFX_RESNET_ZERO1", "0") == "1"
        self.zero1 = bool(zero1) and self.world > 1
        from ..models.resnet import ALIGN

        self.model = ResNet50(device, seed, stages, num_classes,
                              bucket_multiple=ALIGN * (self.world if self.zero1 else 1))
        p = self.model.params
        if self.world > 1:
            from ..ops import transformer as TR

            comm.broadcast_(p.master, 0)
            TR.cast_bf16(p.master, p.bf)
        from ..parallel.comm import make_comm_stream

        self.comm_stream = (make_comm_stream(self.device)
                            if (self.device.type == "cuda" and overlap and self.world > 1) else None)
        # DTFX_RESNET_WSTREAM=1: weight gradients on a second stream (models/resnet.py).  Off:
        # the persistent convolution kernels size their grids for the whole chip, and blocks
        # queued behind a side-stream kernel stretch their tail (10264 vs 10524 img/s, two
        # interleaved rounds, batch 256)
        if self.device.type == "cuda" and os.environ.get("DTFX_RESNET_WSTREAM", "0") == "1":
            self.model.wgrad_stream = torch.cuda.Stream(self.device)
            self.model.wgrad_sync_buckets = self.world > 1
        if (self.device.type == "cuda" and self.world == 1
                and os.environ.get("DTFX_RESNET_FOLD", "1") != "0"):
            # one GPU: SGD sums the split-K weight-gradient planes itself (no reduce launches)
            self.model.enable_splitk_fold()
        self.data = synthetic_imagenet(batch, device, image_size, seed=data_seed,
                                       num_classes=num_classes)
        self.graph = None
        self.last = None
        self.step_count = 0
        if self.zero1:
            p, W, r = self.model.params, self.world, comm.rank
            self._shards = []  # bucket -> (lo, hi, shard lo, shard hi)
            for lo, hi in p.buckets:
                n = (hi - lo) // W
                self._shards.append((lo, hi, lo + r * n, lo + (r + 1) * n))
            gpu = self.device.type == "cuda"
            self._ev_rs = [torch.cuda.Event() if gpu else None for _ in p.buckets]
            self._ev_ag = [torch.cuda.Event() if gpu else None for _ in p.buckets]

    # -- owner-sharded optimizer (ZeRO-1) ------------------------------------------------
    def _gather_bucket(self, b):
        p = self.model.params
        lo, hi, slo, shi = self._shards[b]
        self.comm.all_gather(p.master[lo:hi], p.master[slo:shi])
        self.comm.all_gather(p.bf[lo:hi], p.bf[slo:shi])

    def _zero1_gathers(self):
        """Start of a step: the previous update's shards to every rank (comm stream, forward
        order; block b's forward waits for bucket b only)."""
        if self.comm_stream is None:
            for b in range(len(self._shards)):
                self._gather_bucket(b)
            return
        self.comm_stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.comm_stream):
            for b in range(len(self._shards)):
                self._gather_bucket(b)
                self._ev_ag[b].record(self.comm_stream)

    def _on_needed(self, b):
        if self.comm_stream is not None:
            torch.cuda.current_stream(self.device).wait_event(self._ev_ag[b])

    def _zero1_sgd(self):
        """Momentum SGD of this rank's shards, in the order their reduce-scatters were issued."""
        from ..ops import cnn as CN

        p = self.model.params
        cur = torch.cuda.current_stream(self.device) if self.comm_stream is not None else None
        for b in range(len(self._shards) - 1, -1, -1):
            if cur is not None:
                cur.wait_event(self._ev_rs[b])
            _, _, lo, hi = self._shards[b]
            CN.sgd_momentum_mixed(p.master[lo:hi], p.grad[lo:hi], p.mom[lo:hi], p.bf[lo:hi],
                                  self.lr, self.momentum, self.wd, 1.0 / self.world)
        if cur is not None:
            cur.wait_stream(self.comm_stream)

    def sync_params(self):
        """Complete the non-owned shards after the last update (ZeRO-1): a collective -- every
        rank calls it at the same step.  No-op without sharding."""
        if not self.zero1:
            return
        for b in range(len(self._shards)):
            self._gather_bucket(b)
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()

    def _on_bucket(self, i):
        if self.world == 1:
            return
        if self.zero1:
            p = self.model.params
            lo, hi, slo, shi = self._shards[i]
            if self.comm_stream is None:
                self.comm.reduce_scatter(p.grad[slo:shi], p.grad[lo:hi])
                return
            self.comm_stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.comm_stream):
                self.comm.reduce_scatter(p.grad[slo:shi], p.grad[lo:hi])
                self._ev_rs[i].record(self.comm_stream)
            return
        lo, hi = self.model.params.buckets[i]
        view = self.model.params.grad[lo:hi]
        if self.comm_stream is not None:
            self.comm_stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.comm_stream):
                self.comm.allreduce_sum_(view)
        else:
            self.comm.allreduce_sum_(view)

    def _step_body(self):
        x, y = self.data
        if self.zero1:
            self._zero1_gathers()
            loss, acc = self.model.forward_backward(x, y, on_bucket_ready=self._on_bucket,
                                                    on_bucket_needed=self._on_needed)
            self._zero1_sgd()
            return loss, acc
        loss, acc = self.model.forward_backward(x, y, on_bucket_ready=self._on_bucket)
        if self.comm_stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.comm_stream)
        self.model.sgd_step(self.lr, self.momentum, self.wd, gscale=1.0 / self.world)
        return loss, acc

    def step(self, use_graph=False):
        if not use_graph:
            self.last = self._step_body()
        elif self.graph is None:
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                self.last = self._step_body()
            torch.cuda.current_stream(self.device).wait_stream(s)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self.last = self._step_body()
        else:
            self.graph.replay()
        self.step_count += 1
        return self.last

    def run(self, steps, use_graph=False):
        for _ in range(steps):
            self.step(use_graph)

    def stats(self):
        loss, acc = self.last
        return float(loss.item()), float(acc.item())
