"""BERT-base masked-LM pre-training model on the bf16 gfx950 kernels.

North-star config 5 of BASELINE.json ("BERT-base MLM bf16, bucketed RCCL
all-reduce + fused Adam on 8x MI355X"); the reference itself only trains an
MNIST MLP (worker.py:47-79), so this model follows the public BERT-base
architecture (post-LN encoder, tanh-GELU, tied decoder) rather than any
reference file.

Design (MI355X-first, no autograd graph):

* every parameter lives in ONE flat f32 master buffer (64-element aligned
  slots, forward order), with a flat bf16 working copy used by the GEMMs, one
  flat f32 gradient buffer and the Adam moments -- the optimizer is a single
  fused ``adam_mixed`` launch and each encoder layer's gradients are one
  contiguous all-reduce bucket (7.1 M params = 28 MB, sized for RCCL rings
  over xGMI);
* forward and backward are written out explicitly over the HIP ops
  (``ops.bf16.gemm`` with fused bias/GELU/residual epilogues, fused
  attention, LayerNorm, embedding kernels); backward calls
  ``on_bucket_ready(i)`` as soon as bucket ``i``'s gradients are final, so
  the data-parallel wrapper can start its all-reduce while earlier layers are
  still in backward;
* the QKV projection is one [3H, H] GEMM whose output the attention kernel
  reads in place (no head permutes).

All ops also run on CPU tensors through their f32 reference paths, so a tiny
configuration trains on the CPU test tier.
"""
from __future__ import annotations

import dataclasses
import math
import os

import torch

from ..ops import bf16 as B16
from ..ops import init as I
from ..ops import transformer as TR

BF16 = torch.bfloat16
# DTFX_BERT_WGRAD_BATCH=1: a layer's weight gradients issued to the side stream together after
# its data-gradient chain (one cross-stream edge per layer instead of per GEMM).  Measured
# slower, 7,715-7,726 vs 7,916-7,925 seq/s (profiles/r4/bert/wgrad_batch_ab): the per-GEMM
# edges cost ~15 us of idle GPU each, but starting each weight gradient as soon as its operand
# exists overlaps more of the data-gradient chain.
_WGRAD_BATCH = os.environ.get("DTFX_BERT_WGRAD_BATCH", "0") == "1"
# DTFX_BERT_GELU_DSAVE=1: the FFN input GEMM stores gelu'(u) (from the sigmoid its GELU computes
# anyway) instead of the pre-activation u, so the FFN output dgrad's epilogue is one multiply
# instead of a second exp + rcp + ~8 VALU per element
_GELU_DSAVE = os.environ.get("DTFX_BERT_GELU_DSAVE", "1") == "1"
# DTFX_BERT_BF16_LOGITS=1 (default): the decoder GEMM writes the [masked rows x vocab] logits in
# bf16 (the usual mixed-precision recipe: the cross-entropy still runs in f32 on them), halving
# the 0.3 GB the GEMM writes and the loss reads (+0.2-0.5 %, profiles/r5/bf16_logits/)
_BF16_LOGITS = os.environ.get("DTFX_BERT_BF16_LOGITS", "1") == "1"
ALIGN = 64


@dataclasses.dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    ffn: int = 3072
    max_pos: int = 512
    type_vocab: int = 2
    eps: float = 1e-12
    init_std: float = 0.02

    @property
    def vocab_padded(self):
        return (self.vocab_size + ALIGN - 1) // ALIGN * ALIGN

    @staticmethod
    def base():
        return BertConfig()

    @staticmethod
    def tiny():
        return BertConfig(vocab_size=1000, hidden=128, layers=2, heads=2, ffn=256, max_pos=128)


def param_layout(cfg: BertConfig):
    """[(name, shape, init)] in forward order; init in {"normal", "zeros", "ones"}.

    Weight matrices are [out, in] (GEMM operand op(B) = W^T, TB=1)."""
    H, F, V = cfg.hidden, cfg.ffn, cfg.vocab_padded
    L = [("embeddings/word_embeddings", (V, H), "normal"),
         ("embeddings/position_embeddings", (cfg.max_pos, H), "normal"),
         ("embeddings/token_type_embeddings", (cfg.type_vocab, H), "normal"),
         ("embeddings/LayerNorm/gamma", (H,), "ones"),
         ("embeddings/LayerNorm/beta", (H,), "zeros")]
    for l in range(cfg.layers):
        p = "encoder/layer_%d/" % l
        L += [(p + "attention/qkv/kernel", (3 * H, H), "normal"),
              (p + "attention/qkv/bias", (3 * H,), "zeros"),
              (p + "attention/output/dense/kernel", (H, H), "normal"),
              (p + "attention/output/dense/bias", (H,), "zeros"),
              (p + "attention/output/LayerNorm/gamma", (H,), "ones"),
              (p + "attention/output/LayerNorm/beta", (H,), "zeros"),
              (p + "intermediate/dense/kernel", (F, H), "normal"),
              (p + "intermediate/dense/bias", (F,), "zeros"),
              (p + "output/dense/kernel", (H, F), "normal"),
              (p + "output/dense/bias", (H,), "zeros"),
              (p + "output/LayerNorm/gamma", (H,), "ones"),
              (p + "output/LayerNorm/beta", (H,), "zeros")]
    L += [("cls/predictions/transform/dense/kernel", (H, H), "normal"),
          ("cls/predictions/transform/dense/bias", (H,), "zeros"),
          ("cls/predictions/transform/LayerNorm/gamma", (H,), "ones"),
          ("cls/predictions/transform/LayerNorm/beta", (H,), "zeros"),
          ("cls/predictions/output_bias", (V,), "zeros")]
    return L


class FlatParams:
    """Flat f32 master / bf16 copy / f32 grad / Adam moments with named views.

    ``bucket_multiple`` (a multiple of ALIGN): every gradient bucket's length is padded to a
    multiple of it -- the owner-sharded optimizer (``BertTrainer(zero1=True)``) splits each
    bucket into world-size equal, ALIGN-aligned shards.  The padding stays zero."""

    def __init__(self, cfg: BertConfig, device, seed=0, bucket_multiple=ALIGN):
        self.cfg = cfg
        self.layout = param_layout(cfg)
        self.offsets = {}
        bm = int(bucket_multiple)
        if bm < ALIGN or bm % ALIGN:
            raise ValueError("bucket_multiple must be a positive multiple of %d" % ALIGN)
        starts = {"encoder/layer_%d/attention/qkv/kernel" % l for l in range(cfg.layers)}
        starts.add("cls/predictions/transform/dense/kernel")
        off = 0
        for name, shape, _ in self.layout:
            if name in starts:  # a bucket edge: the previous bucket ends on a multiple
                off = (off + bm - 1) // bm * bm
            n = math.prod(shape)
            self.offsets[name] = (off, shape)
            off += (n + ALIGN - 1) // ALIGN * ALIGN
        off = (off + bm - 1) // bm * bm
        self.numel = off
        dev = torch.device(device)
        self.master = torch.zeros(off, device=dev)
        self.grad = torch.zeros(off, device=dev)
        self.m = torch.zeros(off, device=dev)
        self.v = torch.zeros(off, device=dev)
        self.bf = torch.zeros(off, device=dev, dtype=BF16)
        for i, (name, shape, kind) in enumerate(self.layout):
            t = self.view(self.master, name)
            if kind == "normal":
                I.fill_(t.view(-1), "truncated_normal", 0.0, cfg.init_std, seed=seed, offset=i << 40)
            elif kind == "ones":
                t.fill_(1.0)
        # padded vocabulary rows stay zero (never indexed; masked in the loss)
        w = self.view(self.master, "embeddings/word_embeddings")
        w[cfg.vocab_size:].zero_()
        TR.cast_bf16(self.master, self.bf)
        # buckets: [embeddings, layer 0 .. L-1, head] as contiguous flat ranges
        self.buckets = []
        first = lambda n: self.offsets[n][0]
        lay0 = [first("encoder/layer_%d/attention/qkv/kernel" % l) for l in range(cfg.layers)]
        head0 = first("cls/predictions/transform/dense/kernel")
        edges = [0] + lay0 + [head0, self.numel]
        self.buckets = [(edges[i], edges[i + 1]) for i in range(len(edges) - 1)]

        self._zero_views = None

    # weight gradients that exactly one GEMM writes per step (beta = 0): never zeroed
    @staticmethod
    def overwritten(name):
        # (the word embeddings: the tied decoder's weight-gradient GEMM writes the whole slot
        # with beta = 0 first, the embedding lookup's gradient is added to it afterwards)
        return name.startswith("encoder/") and name.endswith("/kernel") or \
            name in ("cls/predictions/transform/dense/kernel", "embeddings/word_embeddings")

    def zero_grad(self):
        """Zero the gradient slots that the backward ACCUMULATES into (embeddings, biases,
        LayerNorm parameters -- atomics / beta = 1 epilogues) and the alignment padding; the
        GEMM-written weight gradients (``overwritten``) are skipped: 109 of the 110 M slots
        of BERT-base, ~0.44 GB of stores per step (and the tied decoder's gradient GEMM reads no
        zeros: 94 MB less).  The per-layer ranges repeat at the layer
        stride, so each becomes ONE strided view over all layers: a handful of launches."""
        if self._zero_views is None:
            keep, ranges, pos = [], [], 0
            for name, shape, _ in self.layout:
                if self.overwritten(name):
                    off = self.offsets[name][0]
                    keep.append((off, off + math.prod(shape)))
            for a, b in sorted(keep):
                if a > pos:
                    ranges.append((pos, a))
                pos = b
            if pos < self.numel:
                ranges.append((pos, self.numel))
            lay = [self.offsets["encoder/layer_%d/attention/qkv/kernel" % l][0]
                   for l in range(self.cfg.layers)]
            stride = lay[1] - lay[0] if len(lay) > 1 else 0
            periodic = len(lay) > 1 and all(lay[i + 1] - lay[i] == stride for i in range(len(lay) - 1))
            rs, views = set(ranges), []
            for a, b in ranges:
                if (a, b) not in rs:
                    continue  # already covered by a strided view
                rel = a - lay[0]
                if periodic and 0 <= rel < stride and all(
                        (lay[l] + rel, lay[l] + rel + b - a) in rs for l in range(len(lay))):
                    views.append(self.grad.as_strided((len(lay), b - a), (stride, 1), a))
                    for l in range(len(lay)):
                        rs.discard((lay[l] + rel, lay[l] + rel + b - a))
                else:
                    views.append(self.grad[a:b])
                    rs.discard((a, b))
            self._zero_views = views
            self._zero_tab = None
            if self.grad.is_cuda and os.environ.get("DTFX_ZERO_RANGES", "1") != "0":
                # every range in ONE launch (zero_ranges_kernel) instead of a fill per view
                rows, tot = [], 0
                for a, b in sorted(ranges):
                    rows.append((self.grad.data_ptr() + 4 * a, b - a, tot))
                    tot += b - a
                self._zero_tab = (torch.tensor(rows, dtype=torch.int64, device=self.grad.device),
                                  len(rows), tot)
        if self._zero_tab is not None:
            from ..ops._ext import hip, stream_handle

            tab, n, tot = self._zero_tab
            hip().zero_ranges(tab.data_ptr(), n, tot, stream_handle())
            return
        for v in self._zero_views:
            v.zero_()

    def view(self, flat, name):
        off, shape = self.offsets[name]
        return flat[off:off + math.prod(shape)].view(shape)

    def P(self, name):   # f32 master (biases, LayerNorm params)
        return self.view(self.master, name)

    def W(self, name):   # bf16 working copy (GEMM operands, embeddings)
        return self.view(self.bf, name)

    def G(self, name):
        return self.view(self.grad, name)

    def state_dict(self):
        return {n: self.view(self.master, n).detach().cpu() for n, _, _ in self.layout}


class BertMLM:
    """Explicit forward + backward of BERT MLM over the HIP ops."""

    def __init__(self, cfg: BertConfig, device, seed=0, bucket_multiple=ALIGN):
        self.cfg = cfg
        self.device = torch.device(device)
        self.params = FlatParams(cfg, device, seed, bucket_multiple)
        # encoder weight gradients on a second HIP stream: they only need the layer's output
        # gradient and saved input, so they overlap the (independent) dgrad GEMMs -- whose
        # last wave is half empty at M = 16K tokens, N = 768 (768 tiles on 512 resident
        # slots).  ``wgrad_sync_buckets``: join before every gradient-bucket hook (sync DP).
        self.wgrad_stream = None
        self.wgrad_sync_buckets = True
        self._parts = {}     # weight name -> split-K partial planes (enable_splitk_fold)
        self._fold_tokens = None  # the weight gradients' K those planes were sized for
        self._segs = None    # their AdamW segment table

    # ------------------------------------------------------------------ forward
    def _layer_fwd(self, l, x, batch, seq, kmask):
        cfg, p = self.cfg, self.params
        pre = "encoder/layer_%d/" % l
        qkv = B16.gemm(x, p.W(pre + "attention/qkv/kernel"), False, True,
                       bias=p.P(pre + "attention/qkv/bias"))
        ctx, lse = TR.attn_fwd(qkv, batch, seq, cfg.heads, kmask)
        a = B16.gemm(ctx, p.W(pre + "attention/output/dense/kernel"), False, True,
                     bias=p.P(pre + "attention/output/dense/bias"), residual=x)
        h1, m1, r1 = TR.layernorm_fwd(a, p.P(pre + "attention/output/LayerNorm/gamma"),
                                      p.P(pre + "attention/output/LayerNorm/beta"), cfg.eps)
        u = torch.empty(x.shape[0], cfg.ffn, device=x.device, dtype=BF16)
        g = B16.gemm(h1, p.W(pre + "intermediate/dense/kernel"), False, True,
                     bias=p.P(pre + "intermediate/dense/bias"),
                     act="gelu_dsave" if _GELU_DSAVE else "gelu", aux_out=u)
        f = B16.gemm(g, p.W(pre + "output/dense/kernel"), False, True,
                     bias=p.P(pre + "output/dense/bias"), residual=h1)
        out, m2, r2 = TR.layernorm_fwd(f, p.P(pre + "output/LayerNorm/gamma"),
                                       p.P(pre + "output/LayerNorm/beta"), cfg.eps)
        return out, (x, qkv, ctx, lse, a, m1, r1, h1, u, g, f, m2, r2)

    def forward_backward(self, ids, tt, mask_pos, mask_labels, kmask=None, on_bucket_ready=None,
                         n_valid=None, on_bucket_needed=None):
        """One MLM training step's forward + backward; gradients land in params.grad.

        ids, tt: int32 [B, S]; mask_pos: int64 flat token indices of the masked
        positions [Tm]; mask_labels: int32 [Tm].  ``on_bucket_needed(i)``: called before the
        forward first reads bucket ``i``'s parameters (the owner-sharded optimizer's
        all-gather of the previous update is waited for there).  Returns (loss, accuracy) as
        0-dim device tensors (no host sync)."""
        cfg, p = self.cfg, self.params
        batch, seq = ids.shape
        if seq > cfg.max_pos:
            raise ValueError("sequence length %d exceeds max_pos %d" % (seq, cfg.max_pos))
        Tn = batch * seq
        if self._parts and Tn != self._fold_tokens:
            raise ValueError("forward_backward: split-K fold was enabled for %d tokens, this "
                             "batch has %d (call enable_splitk_fold again or disable it)"
                             % (self._fold_tokens, Tn))
        p.zero_grad()
        need = on_bucket_needed if on_bucket_needed is not None else (lambda i: None)
        need(0)
        ids_f, tt_f = ids.reshape(-1), tt.reshape(-1)
        x0, h, me, re = TR.embed_ln_fwd(ids_f, tt_f, p.W("embeddings/word_embeddings"),
                                        p.W("embeddings/position_embeddings"),
                                        p.W("embeddings/token_type_embeddings"),
                                        p.P("embeddings/LayerNorm/gamma"),
                                        p.P("embeddings/LayerNorm/beta"), seq, cfg.eps)
        saved = []
        for l in range(cfg.layers):
            need(l + 1)
            h, s = self._layer_fwd(l, h, batch, seq, kmask)
            saved.append(s)
        # ---- MLM head on the masked positions only
        need(len(p.buckets) - 1)
        hm = h.index_select(0, mask_pos)
        ut = torch.empty(hm.shape, device=h.device, dtype=BF16)
        t = B16.gemm(hm, p.W("cls/predictions/transform/dense/kernel"), False, True,
                     bias=p.P("cls/predictions/transform/dense/bias"), act="gelu", aux_out=ut)
        tn, mt, rt = TR.layernorm_fwd(t, p.P("cls/predictions/transform/LayerNorm/gamma"),
                                      p.P("cls/predictions/transform/LayerNorm/beta"), cfg.eps)
        E = p.W("embeddings/word_embeddings")
        logits = B16.gemm(tn, E, False, True, bias=p.P("cls/predictions/output_bias"),
                          out_dtype=BF16 if _BF16_LOGITS else torch.float32)
        Tm = tn.shape[0]
        scale = 1.0 / max(1, n_valid if n_valid is not None else Tm)
        loss_rows, correct, dlog_b = TR.mlm_xent(logits, mask_labels, cfg.vocab_size, scale)
        loss = loss_rows.sum() * scale
        acc = correct.sum() * scale
        # ---- backward: head
        B16.gemm(dlog_b, tn, True, False, out=p.G("embeddings/word_embeddings"), beta=0.0)
        B16.colsum(dlog_b, out=p.G("cls/predictions/output_bias"), beta=1.0)
        # few output tiles (masked rows x 768) over a deep K (the vocabulary): f32 output so
        # the GEMM can split K over the chip, then one cast (measured 540 -> ~200 us)
        dtn = TR.cast_bf16(B16.gemm(dlog_b, E, out_dtype=torch.float32))
        dt = TR.layernorm_bwd(dtn, t, mt, rt, p.P("cls/predictions/transform/LayerNorm/gamma"),
                              p.G("cls/predictions/transform/LayerNorm/gamma"),
                              p.G("cls/predictions/transform/LayerNorm/beta"))
        dut = TR.act_grad(dt, ut, "gelu")
        B16.gemm(dut, hm, True, False, out=p.G("cls/predictions/transform/dense/kernel"), beta=0.0)
        B16.colsum(dut, out=p.G("cls/predictions/transform/dense/bias"), beta=1.0)
        dhm = B16.gemm(dut, p.W("cls/predictions/transform/dense/kernel"))
        if on_bucket_ready is not None:
            on_bucket_ready(len(p.buckets) - 1)
        dh = torch.zeros(Tn, cfg.hidden, device=h.device, dtype=BF16)
        dh.index_add_(0, mask_pos, dhm)  # padding rows carry zero gradient
        # ---- backward: encoder
        ws, keep = self.wgrad_stream, []  # keep: operands the side stream still reads

        parts = self._parts
        pending = []  # (dy, x, name) of the layer being differentiated (batched wgrad issue)

        def wgrad(dy, xin, name):  # the only writer of these slots: beta = 0 (zero_grad skips them)
            if ws is None:
                B16.gemm(dy, xin, True, False, out=p.G(name), beta=0.0, partials=parts.get(name))
                return
            if _WGRAD_BATCH:
                pending.append((dy, xin, name))
                return
            ws.wait_stream(torch.cuda.current_stream(dy.device))
            with torch.cuda.stream(ws):
                B16.gemm(dy, xin, True, False, out=p.G(name), beta=0.0, partials=parts.get(name))
            keep.append((dy, xin))

        def flush_wgrads():  # (DTFX_BERT_WGRAD_BATCH=1 only)
            if not pending:
                return
            ws.wait_stream(torch.cuda.current_stream(pending[0][0].device))
            with torch.cuda.stream(ws):
                for dy, xin, name in pending:
                    B16.gemm(dy, xin, True, False, out=p.G(name), beta=0.0,
                             partials=parts.get(name))
            keep.extend((dy, xin) for dy, xin, _ in pending)
            pending.clear()

        for l in reversed(range(cfg.layers)):
            dh = self._layer_bwd(l, dh, saved[l], batch, seq, kmask, wgrad)
            flush_wgrads()
            saved[l] = None
            if on_bucket_ready is not None:
                if ws is not None and self.wgrad_sync_buckets:
                    torch.cuda.current_stream(dh.device).wait_stream(ws)
                on_bucket_ready(l + 1)
        # ---- backward: embeddings
        dx0 = TR.layernorm_bwd(dh, x0, me, re, p.P("embeddings/LayerNorm/gamma"),
                               p.G("embeddings/LayerNorm/gamma"), p.G("embeddings/LayerNorm/beta"))
        TR.embed_bwd(ids_f, tt_f, dx0, p.G("embeddings/word_embeddings"),
                     p.G("embeddings/position_embeddings"),
                     p.G("embeddings/token_type_embeddings"), batch, seq)
        if ws is not None:  # join: every gradient final on the main stream
            torch.cuda.current_stream(dx0.device).wait_stream(ws)
            keep.clear()
        if on_bucket_ready is not None:
            on_bucket_ready(0)
        return loss, acc

    def _layer_bwd(self, l, dout, s, batch, seq, kmask, wgrad):
        cfg, p = self.cfg, self.params
        pre = "encoder/layer_%d/" % l
        x, qkv, ctx, lse, a, m1, r1, h1, u, g, f, m2, r2 = s
        # bias gradients are fused into the producer of each activation gradient:
        # LayerNorm bwd (df, da), the act-grad GEMM epilogue (du), attention bwd (dqkv)
        df = TR.layernorm_bwd(dout, f, m2, r2, p.P(pre + "output/LayerNorm/gamma"),
                              p.G(pre + "output/LayerNorm/gamma"), p.G(pre + "output/LayerNorm/beta"),
                              dxsum=p.G(pre + "output/dense/bias"))
        wgrad(df, g, pre + "output/dense/kernel")
        du = B16.gemm(df, p.W(pre + "output/dense/kernel"),  # (u: gelu'(u) under _GELU_DSAVE)
                      act_grad="mul" if _GELU_DSAVE else "gelu", aux_in=u,
                      colsum=p.G(pre + "intermediate/dense/bias"))
        wgrad(du, h1, pre + "intermediate/dense/kernel")
        dh1 = B16.gemm(du, p.W(pre + "intermediate/dense/kernel"), residual=df)
        da = TR.layernorm_bwd(dh1, a, m1, r1, p.P(pre + "attention/output/LayerNorm/gamma"),
                              p.G(pre + "attention/output/LayerNorm/gamma"),
                              p.G(pre + "attention/output/LayerNorm/beta"),
                              dxsum=p.G(pre + "attention/output/dense/bias"))
        wgrad(da, ctx, pre + "attention/output/dense/kernel")
        dctx = B16.gemm(da, p.W(pre + "attention/output/dense/kernel"))
        dqkv = TR.attn_bwd(qkv, ctx, dctx, lse, batch, seq, cfg.heads, kmask,
                           dbias=p.G(pre + "attention/qkv/bias"))
        wgrad(dqkv, x, pre + "attention/qkv/kernel")
        return B16.gemm(dqkv, p.W(pre + "attention/qkv/kernel"), residual=da)

    # ------------------------------------------------------------------ optimizer
    ENCODER_WEIGHTS = ("attention/qkv/kernel", "attention/output/dense/kernel",
                       "intermediate/dense/kernel", "output/dense/kernel")

    def enable_splitk_fold(self, tokens):
        """Leave the encoder weight gradients as split-K partial planes and let AdamW sum them
        (one GPU only: with data parallelism the bucket all-reduce needs the reduced gradient).
        Removes the reduce pass of each split weight-gradient GEMM -- it wrote the f32 gradient
        (28 MB for an FFN weight at seq 128 x batch 128) only for AdamW to read it back.
        ``tokens``: the weight gradients' K (batch x seq).  The planes cost S x the gradient's
        memory (~1.4 GB for BERT-base; 288 GB of HBM).  ``p.grad`` no longer holds these
        gradients: :meth:`materialize_grads` sums them there on demand (tests, debugging)."""
        if not self.device.type == "cuda":
            return 0
        p, rows = self.params, []
        self._parts = {}
        self._fold_tokens = int(tokens)
        for l in range(self.cfg.layers):
            for w in self.ENCODER_WEIGHTS:
                name = "encoder/layer_%d/%s" % (l, w)
                off, (M, N) = p.offsets[name]
                S = B16.splitk_planes(M, N, int(tokens))
                if S <= 1:
                    continue
                buf = torch.zeros(S * M * N, device=self.device)
                self._parts[name] = buf
                rows.append((off // 4, (off + M * N) // 4, buf.data_ptr(), (M * N) // 4, S))
        rows.sort()
        if len(rows) > 128:
            raise ValueError("enable_splitk_fold: at most 128 split weight gradients")
        self._segs = (torch.tensor(rows, dtype=torch.int64, device=self.device)
                      if rows else None)
        # per-bucket tables (adam_step over one bucket's range): built once, graph-safe
        self._seg_rows = rows
        self._bucket_segs = {}
        return len(rows)

    def _segs_for(self, lo, hi):
        if self._segs is None:
            return None
        if (lo, hi) == (0, self.params.numel):
            return self._segs
        key = (lo, hi)
        if key not in self._bucket_segs:
            rows = [r for r in self._seg_rows if r[0] * 4 >= lo and r[1] * 4 <= hi]
            if any(r[0] * 4 < hi and r[1] * 4 > lo and not (r[0] * 4 >= lo and r[1] * 4 <= hi)
                   for r in self._seg_rows):
                raise ValueError("adam_step: range [%d, %d) cuts a folded gradient" % key)
            self._bucket_segs[key] = (torch.tensor(rows, dtype=torch.int64, device=self.device)
                                      if rows else None)
        return self._bucket_segs[key]

    def materialize_grads(self):
        """Sum every folded weight gradient's planes into ``params.grad`` (split order)."""
        p = self.params
        for name, buf in self._parts.items():
            g = p.G(name)
            S = buf.numel() // g.numel()
            planes = buf.view(S, *g.shape)
            acc = planes[0].clone()
            for s in range(1, S):
                acc += planes[s]
            g.copy_(acc)

    def adam_step(self, lr, step, gscale=1.0, wd=0.01, step_ptr=None, lo=0, hi=None):
        """Fused AdamW over the flat range [lo, hi) (default: every parameter); ranges split
        at bucket edges (ALIGN-aligned) give bit-identical results to one launch."""
        p = self.params
        hi = p.numel if hi is None else hi
        sl = slice(lo, hi)
        TR.adam_mixed(p.master[sl], p.grad[sl], p.m[sl], p.v[sl], p.bf[sl], lr, step, wd=wd,
                      gscale=gscale, step_ptr=step_ptr, segs=self._segs_for(lo, hi), base=lo)


MASK_ID = 103  # "[MASK]" in the BERT uncased vocabulary


def _markov_tokens(cfg, n, seq, g, sub_vocab=4096, fanout=4):
    """Token sequences of a sparse first-order Markov chain over a sub-vocabulary: every
    token has ``fanout`` possible successors with skewed probabilities, so a masked token
    is partly predictable from its left neighbour (an MLM signal the model can learn, with
    accuracy well below 1), unlike uniformly random ids."""
    V = min(sub_vocab, cfg.vocab_size - 1000)
    vocab = torch.randperm(cfg.vocab_size - 1000, generator=g)[:V] + 1000  # skip specials
    succ = torch.randint(0, V, (V, fanout), generator=g)
    probs = torch.tensor([0.55, 0.25, 0.12, 0.08][:fanout])
    cur = torch.randint(0, V, (n,), generator=g)
    out = torch.empty(n, seq, dtype=torch.long)
    for t in range(seq):
        out[:, t] = cur
        pick = torch.multinomial(probs, n, replacement=True, generator=g)
        cur = succ[cur, pick]
    return vocab[out].to(torch.int32)


def synthetic_mlm_batch(cfg: BertConfig, batch, seq, device, max_pred=None, seed=0, pad_to=64):
    """One masked-LM batch of the pre-training shape (BERT's recipe on synthetic text).

    Token ids come from a sparse Markov chain (``_markov_tokens``); 15 % of the positions
    (``max_pred``) are selected per sequence and their ORIGINAL ids become the labels; the
    inputs at those positions are replaced by ``[MASK]`` 80 % of the time, a random id
    10 %, kept 10 %.  Returns (ids, tt, mask_pos, labels, n_valid); the masked-position
    list is padded to a multiple of ``pad_to`` with (position 0, label -100) rows."""
    g = torch.Generator().manual_seed(seed)
    max_pred = max_pred or max(1, round(0.15 * seq))
    ids = _markov_tokens(cfg, batch, seq, g) if cfg.vocab_size > 2000 else torch.randint(
        1000 if cfg.vocab_size > 1100 else 0, cfg.vocab_size, (batch, seq), generator=g,
        dtype=torch.int32)
    tt = (torch.arange(seq)[None, :] >= seq // 2).to(torch.int32).expand(batch, seq).contiguous()
    pos = torch.stack([torch.randperm(seq, generator=g)[:max_pred] for _ in range(batch)])
    flat = (pos + torch.arange(batch)[:, None] * seq).reshape(-1)
    ids_flat = ids.reshape(-1)
    labels = ids_flat[flat].clone()
    r = torch.rand(flat.numel(), generator=g)
    rand_ids = torch.randint(0, cfg.vocab_size, (flat.numel(),), generator=g, dtype=torch.int32)
    mask_id = MASK_ID if cfg.vocab_size > MASK_ID else 0
    ids_flat[flat] = torch.where(r < 0.8, torch.full_like(labels, mask_id),
                                 torch.where(r < 0.9, rand_ids, labels))
    n_valid = flat.numel()
    pad = (-n_valid) % pad_to
    if pad:
        flat = torch.cat([flat, torch.zeros(pad, dtype=flat.dtype)])
        labels = torch.cat([labels, torch.full((pad,), -100, dtype=torch.int32)])
    dev = torch.device(device)
    return ids.to(dev), tt.to(dev), flat.to(dev), labels.to(dev), n_valid


def synthetic_mlm_pool(cfg: BertConfig, nbatches, batch, seq, device, seed=0, pad_to=64):
    """``nbatches`` device-resident batches of ``synthetic_mlm_batch`` stacked on a leading
    axis (a rotating dataset: the trainer copies batch k into its step's static buffers)."""
    bs = [synthetic_mlm_batch(cfg, batch, seq, "cpu", seed=seed * 7919 + k, pad_to=pad_to)
          for k in range(nbatches)]
    dev = torch.device(device)
    return tuple(torch.stack([b[i] for b in bs]).to(dev) for i in range(4)), bs[0][4]


# ---------------------------------------------------------------------------
# TF checkpoint naming (google-research/bert layout): kernels [in, out], the
# fused QKV split into query/key/value, the vocabulary unpadded.
# ---------------------------------------------------------------------------
def tf_variables(model: BertMLM):
    """name -> CPU f32 tensor in the original BERT TF checkpoint layout."""
    cfg, p = model.cfg, model.params
    H, V = cfg.hidden, cfg.vocab_size
    m = lambda n: p.P(n).detach().float().cpu()  # noqa: E731
    out = {"bert/embeddings/word_embeddings": m("embeddings/word_embeddings")[:V],
           "bert/embeddings/position_embeddings": m("embeddings/position_embeddings"),
           "bert/embeddings/token_type_embeddings": m("embeddings/token_type_embeddings"),
           "bert/embeddings/LayerNorm/gamma": m("embeddings/LayerNorm/gamma"),
           "bert/embeddings/LayerNorm/beta": m("embeddings/LayerNorm/beta")}
    for l in range(cfg.layers):
        src, dst = "encoder/layer_%d/" % l, "bert/encoder/layer_%d/" % l
        qkv_w, qkv_b = m(src + "attention/qkv/kernel"), m(src + "attention/qkv/bias")
        for i, nm in enumerate(("query", "key", "value")):
            out[dst + "attention/self/%s/kernel" % nm] = qkv_w[i * H:(i + 1) * H].t().contiguous()
            out[dst + "attention/self/%s/bias" % nm] = qkv_b[i * H:(i + 1) * H].clone()
        for a, b in (("attention/output/dense", "attention/output/dense"),
                     ("intermediate/dense", "intermediate/dense"), ("output/dense", "output/dense")):
            out[dst + b + "/kernel"] = m(src + a + "/kernel").t().contiguous()
            out[dst + b + "/bias"] = m(src + a + "/bias")
        for ln in ("attention/output/LayerNorm", "output/LayerNorm"):
            out[dst + ln + "/gamma"] = m(src + ln + "/gamma")
            out[dst + ln + "/beta"] = m(src + ln + "/beta")
    out["cls/predictions/transform/dense/kernel"] = \
        m("cls/predictions/transform/dense/kernel").t().contiguous()
    out["cls/predictions/transform/dense/bias"] = m("cls/predictions/transform/dense/bias")
    out["cls/predictions/transform/LayerNorm/gamma"] = m("cls/predictions/transform/LayerNorm/gamma")
    out["cls/predictions/transform/LayerNorm/beta"] = m("cls/predictions/transform/LayerNorm/beta")
    out["cls/predictions/output_bias"] = m("cls/predictions/output_bias")[:V]
    return out


def load_tf_variables(model: BertMLM, values):
    """Inverse of :func:`tf_variables`; refreshes the bf16 working copy."""
    cfg, p = model.cfg, model.params
    H, V = cfg.hidden, cfg.vocab_size

    def put(name, t):
        dst = p.P(name)
        dst.copy_(torch.as_tensor(t, dtype=torch.float32).reshape(dst.shape).to(dst.device))

    w = p.P("embeddings/word_embeddings")
    w[:V].copy_(torch.as_tensor(values["bert/embeddings/word_embeddings"]).to(w.device))
    for n in ("position_embeddings", "token_type_embeddings", "LayerNorm/gamma", "LayerNorm/beta"):
        put("embeddings/" + n, values["bert/embeddings/" + n])
    for l in range(cfg.layers):
        src, dst = "encoder/layer_%d/" % l, "bert/encoder/layer_%d/" % l
        qkv_w = torch.cat([torch.as_tensor(values[dst + "attention/self/%s/kernel" % nm]).t()
                           for nm in ("query", "key", "value")], 0)
        qkv_b = torch.cat([torch.as_tensor(values[dst + "attention/self/%s/bias" % nm])
                           for nm in ("query", "key", "value")], 0)
        put(src + "attention/qkv/kernel", qkv_w)
        put(src + "attention/qkv/bias", qkv_b)
        for a in ("attention/output/dense", "intermediate/dense", "output/dense"):
            put(src + a + "/kernel", torch.as_tensor(values[dst + a + "/kernel"]).t())
            put(src + a + "/bias", values[dst + a + "/bias"])
        for ln in ("attention/output/LayerNorm", "output/LayerNorm"):
            put(src + ln + "/gamma", values[dst + ln + "/gamma"])
            put(src + ln + "/beta", values[dst + ln + "/beta"])
    put("cls/predictions/transform/dense/kernel",
        torch.as_tensor(values["cls/predictions/transform/dense/kernel"]).t())
    for n in ("transform/dense/bias", "transform/LayerNorm/gamma", "transform/LayerNorm/beta"):
        put("cls/predictions/" + n, values["cls/predictions/" + n])
    ob = p.P("cls/predictions/output_bias")
    ob[:V].copy_(torch.as_tensor(values["cls/predictions/output_bias"]).to(ob.device))
    TR.cast_bf16(p.master, p.bf)
