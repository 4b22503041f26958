"""bf16 matrix-core ops (north-star path: BERT-base, ResNet-50).

GPU tensors run ``csrc/kernels/gemm_bf16.hip`` (v_mfma_f32_16x16x32_bf16,
f32 accumulate, fused epilogues); CPU tensors run an f32 PyTorch reference of
the same math (rounded to the output dtype), which the numerics tests compare
against.  A GPU call with the extension missing raises (no silent fallback).

These ops have no counterpart in the reference (it only runs f32 dense layers,
worker.py:50-53); they serve BASELINE.json's ResNet-50 / BERT-base configs.
"""
from __future__ import annotations

import os

import torch

from ._ext import hip, ptr, stream_handle

# split-K partials through a workspace + reduce pass (DTFX_SPLITK_WS=0: f32 atomics into the output)
_SPLITK_WS = os.environ.get("DTFX_SPLITK_WS", "1") != "0"

ACT = {None: 0, "none": 0, "gelu": 1, "relu": 2}
# act "gelu_dsave" (3): GELU, and ``aux_out`` receives gelu'(pre-activation) instead of the
# pre-activation; act_grad "mul" (3): ``v *= aux_in`` -- the backward of such a forward, one
# multiply per element instead of recomputing the derivative (two transcendentals)
ACT_FWD = dict(ACT, gelu_dsave=3)
ACT_GRAD = dict(ACT, mul=3)


def _gelu_ref(x):
    return torch.nn.functional.gelu(x, approximate="tanh")


def _gelu_grad_ref(u):
    k0, k1 = 0.7978845608028654, 0.044715
    th = torch.tanh(k0 * (u + k1 * u ** 3))
    return 0.5 * (1 + th) + 0.5 * u * (1 - th * th) * k0 * (1 + 3 * k1 * u * u)


def _check(t, name, dtype=torch.bfloat16):
    if t is None:
        return
    if not t.is_cuda:
        raise ValueError("%s must be a GPU tensor" % name)
    if t.dtype != dtype:
        raise TypeError("%s must be %s, got %s" % (name, dtype, t.dtype))
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError("%s must be 2-D with unit column stride" % name)


def gemm(a, b, trans_a=False, trans_b=False, *, bias=None, act=None, aux_out=None, aux_in=None,
         act_grad=None, residual=None, out=None, out_dtype=torch.bfloat16, alpha=1.0, beta=0.0, splitk=0,
         colsum=None, partials=None):
    """``out = epi(alpha * op(a) @ op(b))``, bf16 operands, f32 accumulate.

    Epilogue order: ``+bias`` -> ``aux_out = v`` (pre-activation, bf16) ->
    ``act`` -> ``*= act_grad'(aux_in)`` -> ``+residual`` -> ``+beta*out``.
    ``act`` in {None, "gelu", "relu", "gelu_dsave"}, ``act_grad`` in {None, "gelu", "relu",
    "mul"} (``ACT_FWD`` / ``ACT_GRAD``).  ``splitk`` (0 = auto)
    splits K over workgroups for f32 outputs without epilogue (weight
    gradients: few output tiles, deep K), combining with f32 atomics.
    ``colsum`` (f32 [N]) accumulates the column sums of the final values
    (a fused bias gradient of the produced activation gradient).
    ``partials`` (f32, exactly ``splitk_planes(..) * M * N`` elements): the split-K GEMM leaves
    its S partial planes there and does NOT write ``out`` (no reduce pass): the caller sums them
    (``transformer.adam_mixed(.., segs=..)``).  A GEMM whose split differs from the buffer's
    plane count (or that does not split) raises instead of leaving stale planes.
    """
    act_i = ACT_FWD[act]
    ag_i = ACT_GRAD[act_grad]
    if act_i == 3 and aux_out is None:
        raise ValueError("gemm_bf16: act 'gelu_dsave' stores gelu' in aux_out")
    M = a.shape[1] if trans_a else a.shape[0]
    K = a.shape[0] if trans_a else a.shape[1]
    Kb = b.shape[1] if trans_b else b.shape[0]
    N = b.shape[0] if trans_b else b.shape[1]
    if K != Kb:
        raise ValueError("gemm_bf16: inner dims differ (%d vs %d)" % (K, Kb))
    if out is not None:
        out_dtype = out.dtype
    if not a.is_cuda:
        A = (a.t() if trans_a else a).float()
        B = (b.t() if trans_b else b).float()
        v = alpha * (A @ B)
        if bias is not None:
            v = v + bias.float()
        if act_i == 3:
            aux_out.copy_(_gelu_grad_ref(v))
        elif aux_out is not None:
            aux_out.copy_(v)
        if act_i in (1, 3):
            v = _gelu_ref(v)
        elif act_i == 2:
            v = torch.relu(v)
        if ag_i:
            u = aux_in.float()
            v = v * (u if ag_i == 3 else _gelu_grad_ref(u) if ag_i == 1 else (u > 0).float())
        if residual is not None:
            v = v + residual.float()
        if colsum is not None:
            colsum += v.sum(0)
        if out is not None:
            if beta != 0.0:
                v = v + beta * out.float()
            out.copy_(v)
            return out
        return v.to(out_dtype)
    if K % 64:
        # the kernel consumes K in 64-wide steps: zero-pad both operands along K (small
        # GEMMs only in practice, e.g. a classifier's weight gradient at a small batch)
        Kp = (K + 63) // 64 * 64
        if trans_a:
            a = torch.cat([a, a.new_zeros(Kp - K, a.shape[1])], 0)
        else:
            a = torch.cat([a, a.new_zeros(a.shape[0], Kp - K)], 1)
        if trans_b:
            b = torch.cat([b, b.new_zeros(b.shape[0], Kp - K)], 1)
        else:
            b = torch.cat([b, b.new_zeros(Kp - K, b.shape[1])], 0)
        K = Kp
    _check(a, "a")
    _check(b, "b")
    _check(residual, "residual")
    _check(aux_in, "aux_in")
    _check(aux_out, "aux_out")
    if out is None:
        if beta != 0.0:
            raise ValueError("gemm_bf16: beta != 0 needs out")
        out = torch.empty((M, N), device=a.device, dtype=out_dtype)
    if out.dtype not in (torch.bfloat16, torch.float32):
        raise TypeError("gemm_bf16: out must be bf16 or f32")
    if out.dim() != 2 or out.stride(1) != 1 or tuple(out.shape) != (M, N):
        raise ValueError("gemm_bf16: out must be (%d, %d) with unit column stride" % (M, N))
    if beta != 0.0 and out.dtype != torch.float32:
        raise ValueError("gemm_bf16: beta accumulation needs an f32 out")
    for t, nm in ((aux_in, "aux_in"), (aux_out, "aux_out"), (residual, "residual")):
        if t is not None and tuple(t.shape) != (M, N):
            raise ValueError("gemm_bf16: %s must be (%d, %d)" % (nm, M, N))
    if aux_in is not None and aux_out is not None and aux_in.stride(0) != aux_out.stride(0):
        raise ValueError("gemm_bf16: aux_in/aux_out must share a row stride")
    if ag_i and aux_in is None:
        raise ValueError("gemm_bf16: act_grad needs aux_in")
    if bias is not None:
        if not (bias.is_cuda and bias.dtype == torch.float32 and bias.numel() == N
                and bias.is_contiguous()):
            raise ValueError("gemm_bf16: bias must be a contiguous f32 GPU vector of N elements")
    if colsum is not None and not (colsum.is_cuda and colsum.dtype == torch.float32 and
                                   colsum.numel() == N and colsum.is_contiguous()):
        raise ValueError("gemm_bf16: colsum must be a contiguous f32 GPU vector of N elements")
    aux = aux_in if aux_in is not None else aux_out
    ws, nws = None, 0
    plain = (bias is None and act_i == 0 and ag_i == 0 and residual is None and aux_out is None
             and colsum is None)
    defer = False
    if partials is not None:
        nws = hip().gemm_bf16_ws_floats(bool(trans_a), out.dtype == torch.float32, M, N, K,
                                        int(splitk), float(beta)) if plain else 0
        # the caller sums exactly partials.numel() // (M*N) planes: a GEMM that does not
        # split (nws == 0) or splits into another plane count would leave stale planes there
        if nws != partials.numel():
            raise ValueError("gemm_bf16: this (%d, %d, K=%d) GEMM leaves %d split-K partial "
                             "floats but partials holds %d (split-K fold set up for another "
                             "shape?)" % (M, N, K, nws, partials.numel()))
        if not (partials.is_cuda and partials.dtype == torch.float32
                and partials.is_contiguous()):
            raise ValueError("gemm_bf16: partials must be a contiguous f32 GPU buffer")
        ws, defer = partials, True
    elif out.dtype == torch.float32 and plain and _SPLITK_WS:
        # split-K partials go to a workspace and one reduce pass (plain stores instead of f32
        # atomics, which run at the memory side at ~1.3 TB/s chip-wide)
        nws = hip().gemm_bf16_ws_floats(bool(trans_a), True, M, N, K, int(splitk), float(beta))
        if nws:
            ws = torch.empty(nws, device=a.device, dtype=torch.float32)
    hip().gemm_bf16(bool(trans_a), bool(trans_b), out.dtype == torch.float32, M, N, K,
                    ptr(a), a.stride(0), ptr(b), b.stride(0), ptr(out), out.stride(0),
                    float(alpha), float(beta), ptr(bias), act_i, ptr(aux_in), ptr(aux_out),
                    aux.stride(0) if aux is not None else 0, ptr(residual),
                    residual.stride(0) if residual is not None else 0, ag_i, int(splitk),
                    colsum=ptr(colsum), stream=stream_handle(), ws=ptr(ws), ws_floats=nws,
                    defer_reduce=defer)
    return out


def splitk_planes(M, N, K, trans_a=True, beta=0.0):
    """Split-K planes an f32-output plain GEMM of this shape runs with (1: not split)."""
    nws = hip().gemm_bf16_ws_floats(bool(trans_a), True, M, N, K, 0, float(beta))
    return max(1, nws // (M * N)) if nws else 1


def bmm(a, b, trans_a=False, trans_b=False, *, out=None, out_dtype=torch.bfloat16, alpha=1.0,
        act=None):
    """Strided-batch ``out[i] = act(alpha * op(a[i]) @ op(b[i]))`` for 3-D bf16 tensors
    (each matrix row-major with unit column stride; any batch stride)."""
    if a.dim() != 3 or b.dim() != 3 or a.shape[0] != b.shape[0]:
        raise ValueError("bmm: a and b must be 3-D with equal batch")
    nb = a.shape[0]
    M = a.shape[2] if trans_a else a.shape[1]
    K = a.shape[1] if trans_a else a.shape[2]
    Kb = b.shape[2] if trans_b else b.shape[1]
    N = b.shape[1] if trans_b else b.shape[2]
    if K != Kb:
        raise ValueError("bmm: inner dims differ (%d vs %d)" % (K, Kb))
    if out is not None:
        out_dtype = out.dtype
    if not a.is_cuda:
        A = (a.transpose(1, 2) if trans_a else a).float()
        B = (b.transpose(1, 2) if trans_b else b).float()
        v = alpha * torch.bmm(A, B)
        v = torch.relu(v) if ACT[act] == 2 else (_gelu_ref(v) if ACT[act] == 1 else v)
        if out is not None:
            out.copy_(v)
            return out
        return v.to(out_dtype)
    for t, nm in ((a, "a"), (b, "b")):
        if t.dtype != torch.bfloat16 or t.stride(2) != 1:
            raise ValueError("bmm: %s must be bf16 with unit column stride" % nm)
    if out is None:
        out = torch.empty((nb, M, N), device=a.device, dtype=out_dtype)
    if tuple(out.shape) != (nb, M, N) or out.stride(2) != 1:
        raise ValueError("bmm: out must be (%d, %d, %d) with unit column stride" % (nb, M, N))
    hip().gemm_bf16(bool(trans_a), bool(trans_b), out.dtype == torch.float32, M, N, K,
                    ptr(a), a.stride(1), ptr(b), b.stride(1), ptr(out), out.stride(1),
                    float(alpha), 0.0, 0, ACT[act], 0, 0, 0, 0, 0, 0, 1,
                    batch=nb, sA=a.stride(0), sB=b.stride(0), sC=out.stride(0),
                    stream=stream_handle())
    return out


def colsum(g, out=None, beta=0.0):
    """``out[n] (+)= sum_m g[m, n]`` (bias gradient), bf16 in, f32 out."""
    N = g.shape[1]
    if not g.is_cuda:
        s = g.float().sum(0)
        if out is None:
            return s
        out.copy_(s + beta * out if beta else s)
        return out
    _check(g, "g")
    if out is None:
        if beta != 0.0:
            raise ValueError("colsum: beta needs out")
        out = torch.empty(N, device=g.device, dtype=torch.float32)
    hip().colsum_bf16(ptr(g), g.shape[0], N, g.stride(0), ptr(out), float(beta), stream_handle())
    return out
