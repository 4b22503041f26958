"""Data-parallel ResNet-50 trainer (north-star config 4 of BASELINE.json).

MirroredStrategy-style synchronous SGD: one process per GPU, per-block
gradient buckets all-reduced (sum) on a comm stream as soon as the block's
backward is done, then one fused momentum-SGD launch (f32 master, bf16 copy,
1/world folded in).  The step can be captured in a hipGraph.  The reference
has no counterpart (it trains an MLP with async PS, worker.py:71-79).
"""
from __future__ import annotations

import os

import torch

from ..models.resnet import STAGES, ResNet50, synthetic_imagenet


class ResNetTrainer:
    def __init__(self, batch, device, comm=None, lr=0.1, momentum=0.9, wd=5e-5, seed=0,
                 image_size=224, stages=STAGES, num_classes=1000, overlap=True, data_seed=0):
        self.batch = batch
        self.device = torch.device(device)
        self.comm = comm
        self.world = comm.world_size if comm is not None else 1
        self.lr, self.momentum, self.wd = lr, momentum, wd
        self.model = ResNet50(device, seed, stages, num_classes)
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
        self.data = synthetic_imagenet(batch, device, image_size, seed=data_seed,
                                       num_classes=num_classes)
        self.graph = None
        self.last = None
        self.step_count = 0

    def _on_bucket(self, i):
        if self.world == 1:
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
