"""Transformer ops backed by ``csrc/kernels/transformer.hip`` (gfx950).

GPU tensors run the HIP kernels; CPU tensors run an f32 PyTorch reference of
the same math (used by the CPU tier and by the GPU numerics tests).  There is
no silent fallback for GPU tensors.  North-star BERT-base config of
BASELINE.json; no counterpart in the reference.

Layouts: activations bf16 ``[T, H]`` (T = batch * seq), LayerNorm parameters
and statistics f32, fused QKV activations ``[T, 3 * nh * 64]`` (Q | K | V,
head-major inside each third).
"""
from __future__ import annotations

import math
import os

import torch

from ._ext import hip, ptr, stream_handle

BF16 = torch.bfloat16


def _f(t):
    """f32 view of a low-precision tensor; f32/f64 pass through (reference precision)."""
    return t if t.dtype in (torch.float32, torch.float64) else t.float()


def _contig(t, name, dtype=None):
    if t is None:
        return
    if not t.is_contiguous():
        raise ValueError("%s must be contiguous" % name)
    if dtype is not None and t.dtype != dtype:
        raise TypeError("%s must be %s, got %s" % (name, dtype, t.dtype))


# ---------------------------------------------------------------- LayerNorm
def layernorm_fwd(x, gamma, beta, eps=1e-12):
    T, H = x.shape
    if not x.is_cuda:
        xf = _f(x)
        mean = xf.mean(1)
        rstd = torch.rsqrt(xf.var(1, unbiased=False) + eps)
        y = ((xf - mean[:, None]) * rstd[:, None] * gamma + beta).to(x.dtype)
        return y, mean, rstd
    _contig(x, "x", BF16)
    _contig(gamma, "gamma", torch.float32)
    _contig(beta, "beta", torch.float32)
    y = torch.empty_like(x)
    mean = torch.empty(T, device=x.device)
    rstd = torch.empty(T, device=x.device)
    hip().layernorm_fwd(T, H, ptr(x), ptr(gamma), ptr(beta), float(eps), ptr(y), ptr(mean),
                        ptr(rstd), stream_handle())
    return y, mean, rstd


def layernorm_bwd(dy, x, mean, rstd, gamma, dgamma, dbeta, dres=None, dxsum=None):
    """Returns dx; accumulates dgamma/dbeta (f32) in place, and the column sums of
    dx into ``dxsum`` when given (the next linear layer's bias gradient, fused)."""
    T, H = x.shape
    if not x.is_cuda:
        xf, g = _f(x), _f(dy)
        xh = (xf - mean[:, None]) * rstd[:, None]
        gg = g * gamma
        dx = rstd[:, None] * (gg - gg.mean(1, keepdim=True) - xh * (gg * xh).mean(1, keepdim=True))
        if dres is not None:
            dx = dx + _f(dres)
        dgamma += (g * xh).sum(0)
        dbeta += g.sum(0)
        if dxsum is not None:
            dxsum += dx.sum(0)
        return dx.to(x.dtype)
    for t, n in ((dy, "dy"), (x, "x"), (dres, "dres")):
        _contig(t, n, BF16)
    dx = torch.empty_like(x)
    hip().layernorm_bwd(T, H, ptr(dy), ptr(x), ptr(mean), ptr(rstd), ptr(gamma), ptr(dres),
                        ptr(dx), ptr(dgamma), ptr(dbeta), ptr(dxsum), stream_handle())
    return dx


# ---------------------------------------------------------------- embeddings
def embed_ln_fwd(ids, tt, word, pos, type_, gamma, beta, seq_len, eps=1e-12):
    """x = word[ids] + pos[t % S] + type[tt]; returns (x bf16, LN(x), mean, rstd)."""
    T = ids.numel()
    H = word.shape[1]
    if seq_len > pos.shape[0] or T % seq_len:
        raise ValueError("embed_ln_fwd: seq_len %d vs %d positions / %d tokens"
                         % (seq_len, pos.shape[0], T))
    if not ids.is_cuda:
        p = torch.arange(T) % seq_len
        x = (word[ids.long()].float() + pos[p].float() +
             type_[(tt if tt is not None else torch.zeros_like(ids)).long()].float()).to(word.dtype)
        y, mean, rstd = layernorm_fwd(x, gamma, beta, eps)
        return x, y, mean, rstd
    _contig(ids, "ids", torch.int32)
    _contig(tt, "tt", torch.int32)
    for t, n in ((word, "word"), (pos, "pos"), (type_, "type")):
        _contig(t, n, BF16)
    x = torch.empty(T, H, device=ids.device, dtype=BF16)
    y = torch.empty_like(x)
    mean = torch.empty(T, device=ids.device)
    rstd = torch.empty(T, device=ids.device)
    hip().embed_ln_fwd(T, seq_len, H, ptr(ids), ptr(tt), ptr(word), ptr(pos), ptr(type_),
                       ptr(gamma), ptr(beta), float(eps), ptr(x), ptr(y), ptr(mean), ptr(rstd),
                       stream_handle())
    return x, y, mean, rstd


def embed_bwd(ids, tt, dx, dword, dpos, dtype_, batch, seq_len):
    """Accumulates word / position / token-type gradients (f32) in place."""
    if not dx.is_cuda:
        g = dx.float()
        dword.index_add_(0, ids.long().view(-1), g)
        dpos[:seq_len] += g.view(batch, seq_len, -1).sum(0)
        t = (tt if tt is not None else torch.zeros_like(ids)).long().view(-1)
        dtype_.index_add_(0, t, g)
        return
    _contig(dx, "dx", BF16)
    hip().embed_bwd(batch, seq_len, dx.shape[1], ptr(ids), ptr(tt), ptr(dx), ptr(dword),
                    ptr(dpos), ptr(dtype_), stream_handle())


# ---------------------------------------------------------------- attention
def _split(qkv, batch, seq, nh):
    d = 64
    q, k, v = qkv.float().view(batch, seq, 3, nh, d).permute(2, 0, 3, 1, 4)
    return q, k, v  # [B, nh, S, d]


def _use_flash(seq):
    """S <= 128: whole (sequence, head) in one workgroup's LDS (attn_*_kernel); longer
    sequences: flash-style tiles (flash_attn.hip).  DTFX_ATTN=flash forces the latter."""
    return seq > 128 or os.environ.get("DTFX_ATTN") == "flash"


def lse_ld(seq):
    return max(128, (seq + 63) // 64 * 64)


def attn_fwd(qkv, batch, seq, nh, kmask=None, scale=None):
    """softmax(Q K^T * scale + kmask) V per (sequence, head); returns (out [T, nh*64], lse)
    with lse f32 [batch * nh, lse_ld(seq)]."""
    scale = 1.0 / math.sqrt(64) if scale is None else scale
    if not qkv.is_cuda:
        q, k, v = _split(qkv, batch, seq, nh)
        s = q @ k.transpose(-1, -2) * scale
        if kmask is not None:
            s = s + kmask.view(batch, 1, 1, seq)
        lse = torch.logsumexp(s, -1)
        lse = torch.nn.functional.pad(lse, (0, lse_ld(seq) - seq)).reshape(batch * nh, -1)
        p = torch.softmax(s, -1).to(BF16).float()
        o = (p @ v).permute(0, 2, 1, 3).reshape(batch * seq, nh * 64).to(BF16)
        return o, lse
    _contig(qkv, "qkv", BF16)
    _contig(kmask, "kmask", torch.float32)
    out = torch.empty(batch * seq, nh * 64, device=qkv.device, dtype=BF16)
    lse = torch.empty(batch * nh, lse_ld(seq), device=qkv.device)
    if _use_flash(seq):
        hip().flash_fwd(batch, seq, nh, ptr(qkv), ptr(out), ptr(lse), lse.shape[1], ptr(kmask),
                        float(scale), stream_handle())
    else:
        hip().attn_fwd(batch, seq, nh, ptr(qkv), ptr(out), ptr(lse), ptr(kmask), float(scale),
                       stream_handle())
    return out, lse


def attn_bwd(qkv, o, dout, lse, batch, seq, nh, kmask=None, scale=None, dbias=None):
    """Gradient w.r.t. the fused QKV activations, same layout as ``qkv``; adds its
    column sums (the QKV bias gradient) into ``dbias`` when given."""
    scale = 1.0 / math.sqrt(64) if scale is None else scale
    if not qkv.is_cuda:
        q, k, v = _split(qkv, batch, seq, nh)
        do = dout.float().view(batch, seq, nh, 64).permute(0, 2, 1, 3)
        of = o.float().view(batch, seq, nh, 64).permute(0, 2, 1, 3)
        s = q @ k.transpose(-1, -2) * scale
        if kmask is not None:
            s = s + kmask.view(batch, 1, 1, seq)
        lse_ = lse.view(batch, nh, -1)[..., :seq]
        p = torch.exp(s - lse_[..., None])
        D = (do * of).sum(-1, keepdim=True)
        dp = do @ v.transpose(-1, -2)
        ds = p * (dp - D)
        dv = p.transpose(-1, -2) @ do
        dk = ds.transpose(-1, -2) @ q * scale
        dq = ds @ k * scale
        g = torch.stack([dq, dk, dv], 0)  # [3, B, nh, S, d]
        g = g.permute(1, 3, 0, 2, 4).reshape(batch * seq, 3 * nh * 64)
        if dbias is not None:
            dbias += g.sum(0)
        return g.to(BF16)
    for t, n in ((qkv, "qkv"), (o, "o"), (dout, "dout")):
        _contig(t, n, BF16)
    dqkv = torch.empty_like(qkv)
    if _use_flash(seq):
        scratch = torch.empty_like(lse)
        hip().flash_bwd(batch, seq, nh, ptr(qkv), ptr(o), ptr(dout), ptr(lse), lse.shape[1],
                        ptr(kmask), float(scale), ptr(dqkv), ptr(dbias), ptr(scratch),
                        stream_handle())
    else:
        hip().attn_bwd(batch, seq, nh, ptr(qkv), ptr(o), ptr(dout), ptr(lse), ptr(kmask),
                       float(scale), ptr(dqkv), ptr(dbias), stream_handle())
    return dqkv


# ---------------------------------------------------------------- optimizer / casts
def adam_mixed(p, g, m, v, pb, lr, step, b1=0.9, b2=0.999, eps=1e-6, wd=0.01, gscale=1.0,
               step_ptr=None, segs=None, base=0):
    """AdamW on an f32 master buffer; refreshes the bf16 working copy ``pb``.  ``segs``
    (int64 [nseg, 5] on the GPU, see ``BertMLM.enable_splitk_fold``): flat ranges whose
    gradient is read as the sum of split-K partial planes instead of from ``g``; their bounds
    are offsets into the whole flat buffer, of which ``p``... start at element ``base``."""
    if segs is not None and not p.is_cuda:
        raise ValueError("adam_mixed: segments are a GPU path")
    if not p.is_cuda:
        gg = g * gscale
        m.mul_(b1).add_((1 - b1) * gg)
        v.mul_(b2).add_((1 - b2) * gg * gg)
        t = int(step_ptr.item()) if step_ptr is not None else step
        bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
        p.mul_(1 - lr * wd)
        p.sub_(lr / bc1 * m / (v.sqrt() / math.sqrt(bc2) + eps))
        if pb is not None:
            pb.copy_(p)
        return
    if segs is not None and not (segs.is_cuda and segs.dtype == torch.int64
                                 and segs.is_contiguous() and segs.dim() == 2
                                 and segs.shape[1] == 5):
        raise ValueError("adam_mixed: segs must be a contiguous int64 [nseg, 5] GPU tensor")
    hip().adam_mixed(p.numel(), ptr(p), ptr(g), ptr(m), ptr(v), ptr(pb), float(lr), float(b1),
                     float(b2), float(eps), float(wd), float(gscale), ptr(step_ptr), int(step),
                     stream_handle(), ptr(segs), 0 if segs is None else int(segs.shape[0]),
                     int(base) // 4)


def cast_bf16(x, out=None):
    if out is None:
        out = torch.empty(x.shape, device=x.device, dtype=BF16)
    if not x.is_cuda:
        out.copy_(x)
        return out
    hip().cast_f32_bf16(x.numel(), ptr(x), ptr(out), stream_handle())
    return out


def act_grad(dy, u, act="gelu"):
    """dy * act'(u) for bf16 tensors (act in {"gelu", "relu"})."""
    a = {"gelu": 1, "relu": 2}[act]
    if not dy.is_cuda:
        uf = _f(u)
        if a == 1:
            k0, k1 = 0.7978845608028654, 0.044715
            th = torch.tanh(k0 * (uf + k1 * uf ** 3))
            d = 0.5 * (1 + th) + 0.5 * uf * (1 - th * th) * k0 * (1 + 3 * k1 * uf * uf)
        else:
            d = (uf > 0).to(uf.dtype)
        return (_f(dy) * d).to(dy.dtype)
    _contig(dy, "dy", BF16)
    _contig(u, "u", BF16)
    dx = torch.empty_like(dy)
    hip().act_grad_bf16(dy.numel(), a, ptr(dy), ptr(u), ptr(dx), stream_handle())
    return dx


def mlm_xent(logits, labels, n_classes, scale):
    """Softmax cross-entropy over the first ``n_classes`` columns of f32 or bf16 ``logits``
    [N, ldl] (f32 math either way); labels int32 (-100 = ignore).  Returns (loss_rows, correct_rows,
    dlogits bf16 [N, ldl] pre-scaled by ``scale``, zero beyond n_classes)."""
    N, ldl = logits.shape
    if not logits.is_cuda:
        from .nn import softmax_xent_stats

        loss, d, correct = softmax_xent_stats(logits[:, :n_classes].float(), labels,
                                              want_grad=True, scale=scale)
        dl = torch.zeros(N, ldl, dtype=BF16)
        dl[:, :n_classes] = d.to(BF16)
        return loss, correct, dl
    _contig(logits, "logits", logits.dtype if logits.dtype == BF16 else torch.float32)
    lab = labels.to(torch.int32).contiguous()
    loss = torch.empty(N, device=logits.device)
    correct = torch.empty(N, device=logits.device)
    dl = torch.empty(N, ldl, device=logits.device, dtype=BF16)
    hip().mlm_xent(N, n_classes, ptr(logits), ldl, ptr(lab), float(scale), ptr(loss), ptr(correct),
                   ptr(dl), ldl, stream_handle(), logits.dtype == BF16)
    return loss, correct, dl
