"""Data-parallel BERT-base MLM trainer (north-star config 5 of BASELINE.json).

One process per GPU.  Per step: explicit forward/backward
(``models.bert.BertMLM``); as soon as an encoder layer's backward is done its
gradient bucket (one contiguous 28 MB slice of the flat f32 gradient) is
all-reduced (sum) on a dedicated comm stream, overlapping the remaining
backward; then one fused mixed-precision AdamW launch over the whole flat
buffer (gradient averaging folded in as ``gscale = 1/world``) refreshes the
f32 master weights and the bf16 working copy.  The whole step can be
captured into one hipGraph (``use_graph``): the RCCL calls of the native
communicator are graph-capturable.

Owner-sharded optimizer (``zero1``, the world > 1 default; DTFX_BERT_ZERO1=0 turns it off):
the reference applies every gradient ONCE, on the ps task that owns the variable
(``apply_gradients`` colocated with the variable, worker.py:75-79, placed by
``replica_device_setter``, worker.py:24-25).  Here every GPU owns an equal 1/W shard of each
encoder-layer / head bucket (ZeRO-1):

    backward      bucket i final -> reduce-scatter on the comm stream (half an all-reduce's
                  bytes): this rank holds the summed gradient of its shard
    after it      fused AdamW on the shard only (1/W of the work; Adam moments sized for
                  the shard), in the order the buckets became ready
    next step     all-gather of the shards (f32 master + bf16 working copy) on the comm
                  stream at the start of the step; the forward of layer l waits only for
                  bucket l's gather, so the gathers overlap the forward of the layers below

The embedding bucket (the last one backward produces and the first one forward needs) stays
all-reduced with a replicated AdamW: sharding it would expose its gather at the start of the
forward.  Between steps the non-owned shards of ``params.master`` / ``params.bf`` are one
update behind: ``sync_params()`` (a collective, every rank at the same step) completes them
for checkpoints, evals and replica checks.

Reference counterpart: the reference only has async-PS SGD of an MLP
(worker.py:71-79, 129-159); this is the sync all-reduce design the
BASELINE.json north star asks for, applied to BERT-base.
"""
from __future__ import annotations

import os

import torch

from ..models.bert import BertConfig, BertMLM, synthetic_mlm_pool
from ..ops import optim as OPT


class BertTrainer:
    def __init__(self, cfg: BertConfig, batch, seq, device, comm=None, lr=1e-4, seed=0,
                 overlap=True, weight_decay=0.01, data_seed=None, data_batches=8, zero1=None):
        self.cfg, self.batch, self.seq = cfg, batch, seq
        self.device = torch.device(device)
        self.comm = comm
        self.world = comm.world_size if comm is not None else 1
        self.lr, self.wd = lr, weight_decay
        if zero1 is None:
            zero1 = self.world > 1 and os.environ.get("DTFX_BERT_ZERO1", "1") != "0"
        self.zero1 = bool(zero1) and self.world > 1
        from ..models.bert import ALIGN

        self.model = BertMLM(cfg, device, seed,
                             bucket_multiple=ALIGN * (self.world if self.zero1 else 1))
        p = self.model.params
        if self.world > 1:  # replicas start identical (Philox init is seed-determined; broadcast anyway)
            comm.broadcast_(p.master, 0)
            from ..ops import transformer as TR

            TR.cast_bf16(p.master, p.bf)
        self.gpu = self.device.type == "cuda"
        from ..parallel.comm import make_comm_stream

        self.comm_stream = (make_comm_stream(self.device) if (self.gpu and overlap and self.world > 1)
                            else None)
        # weight gradients on a second stream: on one GPU the step measured 1.7 % faster without
        # it once the attention backward ran two blocks per CU (7,903-7,919 -> 8,034-8,055
        # seq/s, profiles/r4/bert/half_nows/), so it is the multi-GPU default only;
        # DTFX_BERT_WSTREAM=0 / 1 forces it
        ws_env = os.environ.get("DTFX_BERT_WSTREAM")
        if self.gpu and (ws_env == "1" or (ws_env is None and self.world > 1)):
            self.model.wgrad_stream = torch.cuda.Stream(self.device)
            self.model.wgrad_sync_buckets = self.world > 1
        if (self.gpu and self.world == 1 and os.environ.get("DTFX_BERT_FOLD", "1") != "0"
                and (batch * seq) % 64 == 0):
            # one GPU: no all-reduce between the weight gradients and AdamW -> AdamW sums the
            # split-K planes itself (no reduce pass per split weight-gradient GEMM)
            self.model.enable_splitk_fold(batch * seq)
        # a rotating dataset of `data_batches` device-resident MLM batches: before every step
        # (eager or graph replay) batch k is copied into the static buffers the step reads
        self.pool, nv = synthetic_mlm_pool(cfg, data_batches, batch, seq, device,
                                           seed=(data_seed if data_seed is not None else 17))
        self.data = tuple(t[0].clone() for t in self.pool) + (nv,)
        # the embedding bucket (0) is the LAST gradient backward produces: its all-reduce
        # (94 MB of f32 word-embedding gradient for BERT-base) is the one exchange that
        # nothing overlaps, so AdamW of every other bucket runs while it is in flight
        self._body_reduced = (torch.cuda.Event() if self.comm_stream is not None else None)
        # one GPU, DTFX_BERT_OPT_OVERLAP=1 (opt-in): each bucket's AdamW on a third stream as
        # soon as the bucket is final, overlapping the backward of the layers below.  Measured
        # SLOWER (bench.py --model bert: 7,779-7,801 vs 7,859-7,870 seq/s, same box,
        # profiles/r4/bert/): the memory-bound AdamW blocks take CUs and HBM bandwidth from the
        # dgrad / wgrad GEMMs on the critical path, costing more than the 0.66 ms it hides
        self.opt_stream = (torch.cuda.Stream(self.device)
                           if (self.gpu and self.world == 1
                               and os.environ.get("DTFX_BERT_OPT_OVERLAP", "0") == "1") else None)
        self._adam_kw = None
        if self.zero1:
            self._init_zero1()
        self.step_t = torch.ones(1, dtype=torch.int32, device=self.device)  # Adam step (device side)
        self.step_count = 0
        self.graph = None
        self.last = None

    # -- owner-sharded optimizer (ZeRO-1) ------------------------------------------------
    def _init_zero1(self):
        p, W = self.model.params, self.world
        r = self.comm.rank
        self._shards = {}  # bucket -> (lo, hi, shard lo, shard hi, offset in the moment buffers)
        off = 0
        for b, (lo, hi) in enumerate(p.buckets):
            if b == 0:
                continue  # embeddings: all-reduced, replicated AdamW
            n = (hi - lo) // W
            self._shards[b] = (lo, hi, lo + r * n, lo + (r + 1) * n, off)
            off += n
        self._m_sh = torch.zeros(off, device=self.device)
        self._v_sh = torch.zeros(off, device=self.device)
        lo0, hi0 = p.buckets[0]
        self._m_emb = torch.zeros(hi0 - lo0, device=self.device)
        self._v_emb = torch.zeros(hi0 - lo0, device=self.device)
        p.m = p.v = None  # the full-size moments are not kept: 1/W of them per rank
        gpu = self.gpu
        self._ev_rs = {b: (torch.cuda.Event() if gpu else None) for b in range(len(p.buckets))}
        self._ev_ag = {b: (torch.cuda.Event() if gpu else None) for b in self._shards}

    def _gather_bucket(self, b):
        """All-gather bucket b's shards (f32 master + bf16 working copy) on the current stream."""
        p = self.model.params
        lo, hi, slo, shi, _ = self._shards[b]
        self.comm.all_gather(p.master[lo:hi], p.master[slo:shi])
        self.comm.all_gather(p.bf[lo:hi], p.bf[slo:shi])

    def _zero1_gathers(self):
        """Start of a step: the previous update's shards to every rank (comm stream)."""
        if self.comm_stream is None:
            for b in self._shards:
                self._gather_bucket(b)
            return
        cur = torch.cuda.current_stream(self.device)
        self.comm_stream.wait_stream(cur)
        with torch.cuda.stream(self.comm_stream):
            for b in sorted(self._shards):  # forward order: layers, then the head
                self._gather_bucket(b)
                self._ev_ag[b].record(self.comm_stream)

    def _on_needed(self, b):
        if self.comm_stream is not None and b in self._ev_ag:
            torch.cuda.current_stream(self.device).wait_event(self._ev_ag[b])

    def _zero1_bucket(self, i):
        p = self.model.params
        lo, hi = p.buckets[i]
        g = p.grad[lo:hi]

        def issue():
            if i in self._shards:
                _, _, slo, shi, _ = self._shards[i]
                self.comm.reduce_scatter(p.grad[slo:shi], g)
            else:
                self.comm.allreduce_sum_(g)

        if self.comm_stream is None:
            issue()
            return
        self.comm_stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.comm_stream):
            issue()
            self._ev_rs[i].record(self.comm_stream)

    def _zero1_adam(self, kw):
        """AdamW of this rank's shards (in the order their reduce-scatters were issued), then
        the replicated embeddings."""
        from ..ops import transformer as TR

        p = self.model.params
        cur = torch.cuda.current_stream(self.device) if self.comm_stream is not None else None
        order = sorted(self._shards, reverse=True) + [0]
        for b in order:
            if cur is not None:
                cur.wait_event(self._ev_rs[b])
            if b == 0:
                lo, hi = p.buckets[0]
                m, v = self._m_emb, self._v_emb
            else:
                _, _, lo, hi, o = self._shards[b]
                m, v = self._m_sh[o:o + hi - lo], self._v_sh[o:o + hi - lo]
            TR.adam_mixed(p.master[lo:hi], p.grad[lo:hi], m, v, p.bf[lo:hi], self.lr, 0,
                          wd=kw["wd"], gscale=kw["gscale"], step_ptr=kw["step_ptr"])
        if cur is not None:
            cur.wait_stream(self.comm_stream)

    def sync_params(self):
        """Complete the non-owned shards of the parameters after the last update (ZeRO-1): a
        collective -- every rank calls it at the same step.  No-op without sharding."""
        if not self.zero1:
            return
        for b in sorted(self._shards):
            self._gather_bucket(b)
        if self.gpu:
            torch.cuda.current_stream(self.device).synchronize()

    # gradient bucket ready -> all-reduce on the comm stream (one GPU: its AdamW)
    def _on_bucket(self, i):
        if self.zero1:
            return self._zero1_bucket(i)
        if self.world == 1:
            if self.opt_stream is not None and i != 0:  # the embeddings' AdamW: after the join
                lo, hi = self.model.params.buckets[i]
                cur = torch.cuda.current_stream(self.device)
                self.opt_stream.wait_stream(cur)
                if self.model.wgrad_stream is not None:  # the bucket's weight gradients
                    self.opt_stream.wait_stream(self.model.wgrad_stream)
                with torch.cuda.stream(self.opt_stream):
                    self.model.adam_step(self.lr, 0, lo=lo, hi=hi, **self._adam_kw)
            return
        lo, hi = self.model.params.buckets[i]
        view = self.model.params.grad[lo:hi]
        if self.comm_stream is not None:
            self.comm_stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.comm_stream):
                self.comm.allreduce_sum_(view)
                if i == 1:  # the last non-embedding bucket (layer 0): the body is reduced
                    self._body_reduced.record(self.comm_stream)
        else:
            self.comm.allreduce_sum_(view)

    def _step_body(self):
        ids, tt, pos, lab, nv = self.data
        kw = dict(gscale=1.0 / self.world, wd=self.wd, step_ptr=self.step_t)
        self._adam_kw = kw
        if self.zero1:
            self._zero1_gathers()
            loss, acc = self.model.forward_backward(ids, tt, pos, lab, n_valid=nv,
                                                    on_bucket_ready=self._on_bucket,
                                                    on_bucket_needed=self._on_needed)
            self._zero1_adam(kw)
            OPT.counter_add_(self.step_t, 1)
            return loss, acc
        loss, acc = self.model.forward_backward(ids, tt, pos, lab, n_valid=nv,
                                                on_bucket_ready=self._on_bucket)
        if self.opt_stream is not None:
            cur = torch.cuda.current_stream(self.device)
            lo, hi = self.model.params.buckets[0]
            self.model.adam_step(self.lr, 0, lo=lo, hi=hi, **kw)  # embeddings, last bucket
            cur.wait_stream(self.opt_stream)                      # every other bucket's AdamW
        elif self.comm_stream is not None:
            cur = torch.cuda.current_stream(self.device)
            split = self.model.params.buckets[1][0]  # [0, split): embeddings bucket
            cur.wait_event(self._body_reduced)
            self.model.adam_step(self.lr, 0, lo=split, **kw)   # overlaps the embedding all-reduce
            cur.wait_stream(self.comm_stream)
            self.model.adam_step(self.lr, 0, hi=split, **kw)
        else:
            self.model.adam_step(self.lr, 0, **kw)
        OPT.counter_add_(self.step_t, 1)
        return loss, acc

    def _load_batch(self):
        k = self.step_count % self.pool[0].shape[0]
        for dst, src in zip(self.data[:4], self.pool):
            dst.copy_(src[k], non_blocking=True)

    def step(self, use_graph=False):
        self._load_batch()
        if not use_graph:
            self.last = self._step_body()
        elif self.graph is None:
            # this call's step runs eagerly on a side stream (warms the allocator and
            # the kernels' one-time attributes); the same body is then captured once
            # and every later call replays it
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

    def flops_per_step(self):
        """Model FLOPs per step on this rank (6 * matmul params * tokens + attention)."""
        c = self.cfg
        T = self.batch * self.seq
        Tm = self.data[2].numel()
        layer = 2 * T * (3 * c.hidden * c.hidden + c.hidden * c.hidden + 2 * c.hidden * c.ffn)
        attn = 2 * 2 * self.batch * c.heads * self.seq * self.seq * 64
        head = 2 * Tm * (c.hidden * c.hidden + c.hidden * c.vocab_padded)
        return 3 * (c.layers * (layer + attn) + head)
