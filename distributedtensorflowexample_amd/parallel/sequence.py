"""Ulysses sequence parallelism for the BERT attention core.

Not in the reference (its model has no sequence dimension, worker.py:47).
SURVEY.md §5.7 names the xGMI-native choice if sequence parallelism is
added: an all-to-all across <= 8 GPUs, which full-bisection point-to-point
xGMI makes cheap (every pair of GPUs has its own link, so an all-to-all
moves 1/P of each rank's bytes over each link in parallel).

Each of P ranks holds a contiguous 1/P of every sequence (tokens
``[r*S/P, (r+1)*S/P)``) in the fused-QKV layout of ``ops.transformer``
(``[B*S/P, 3*nh*64]``, columns ``[3][nh][64]``).

    forward:   all-to-all  seq-sharded QKV -> head-sharded QKV of the FULL
               sequence (nh/P heads per rank)
               attention kernel (attn_fwd: LDS kernel S<=128, flash above)
               all-to-all  head-sharded O -> seq-sharded O
    backward:  the same two exchanges around attn_bwd, mirrored

Two all-to-alls of activation size per direction; the attention itself sees
whole sequences, so no ring passes or online-softmax merges across ranks are
needed and the result is exactly the single-GPU attention.
"""
from __future__ import annotations

import torch

from ..ops import transformer as T


def _seq_to_head(x, comm, batch, s_loc, groups, nh):
    """[B*S/P, groups*nh*64] seq-sharded -> [B*S, groups*(nh/P)*64] head-sharded."""
    P = comm.world_size
    hp = nh // P
    send = (x.view(batch, s_loc, groups, P, hp, 64).permute(3, 0, 1, 2, 4, 5).contiguous())
    recv = torch.empty_like(send)  # [P (seq chunk = source rank), B, S/P, G, hp, 64]
    comm.all_to_all(recv.view(P, -1), send.view(P, -1))
    return recv.permute(1, 0, 2, 3, 4, 5).reshape(batch * P * s_loc, groups * hp * 64)


def _head_to_seq(y, comm, batch, s_loc, groups, nh):
    """[B*S, groups*(nh/P)*64] head-sharded -> [B*S/P, groups*nh*64] seq-sharded."""
    P = comm.world_size
    hp = nh // P
    send = y.view(batch, P, s_loc, groups, hp, 64).permute(1, 0, 2, 3, 4, 5).contiguous()
    recv = torch.empty_like(send)  # [P (head group = source rank), B, S/P, G, hp, 64]
    comm.all_to_all(recv.view(P, -1), send.view(P, -1))
    return recv.permute(1, 2, 3, 0, 4, 5).reshape(batch * s_loc, groups * nh * 64)


class _UlyssesAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, comm, batch, s_loc, nh, kmask, scale):
        qkv_h = _seq_to_head(qkv, comm, batch, s_loc, 3, nh)
        seq = s_loc * comm.world_size
        o_h, lse = T.attn_fwd(qkv_h, batch, seq, nh // comm.world_size, kmask, scale)
        ctx.save_for_backward(qkv_h, o_h, lse)
        ctx.meta = (comm, batch, s_loc, nh, kmask, scale)
        return _head_to_seq(o_h, comm, batch, s_loc, 1, nh)

    @staticmethod
    def backward(ctx, dout):
        qkv_h, o_h, lse = ctx.saved_tensors
        comm, batch, s_loc, nh, kmask, scale = ctx.meta
        dout_h = _seq_to_head(dout.to(o_h.dtype).contiguous(), comm, batch, s_loc, 1, nh)
        seq = s_loc * comm.world_size
        dqkv_h = T.attn_bwd(qkv_h, o_h, dout_h, lse, batch, seq, nh // comm.world_size, kmask,
                            scale)
        return _head_to_seq(dqkv_h, comm, batch, s_loc, 3, nh), None, None, None, None, None, None


def ulysses_attention(qkv, comm, batch, seq_local, nh, kmask=None, scale=None):
    """Attention over sequences split across ``comm.world_size`` ranks.

    ``qkv``: this rank's tokens, ``[batch*seq_local, 3*nh*64]`` bf16 (fused QKV layout);
    ``kmask``: additive key mask of the FULL sequence, ``[batch, seq_local*P]`` f32 (the
    same on every rank) or None.  Returns ``[batch*seq_local, nh*64]`` bf16, equal to the
    rows of single-device attention over the whole sequence that this rank holds.
    """
    P = comm.world_size
    if nh % P:
        raise ValueError("Ulysses SP needs heads (%d) divisible by the SP degree (%d)" % (nh, P))
    if qkv.shape != (batch * seq_local, 3 * nh * 64):
        raise ValueError("qkv shape %s != [%d, %d]" % (tuple(qkv.shape), batch * seq_local,
                                                       3 * nh * 64))
    return _UlyssesAttention.apply(qkv.contiguous(), comm, batch, seq_local, nh, kmask, scale)


__all__ = ["ulysses_attention"]
