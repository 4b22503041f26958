"""Dense-layer and loss ops backed by the gfx950 kernels.

GPU tensors run the hand-written HIP kernels (``csrc/kernels``); CPU tensors
run an explicit PyTorch reference of the same math (CPU tier / plumbing
config).  There is no silent GPU fallback: a GPU call with the extension
missing raises.

Ops (TF 1.x counterparts used by the reference, worker.py:46-79):

* :func:`gemm`           -- MatMul (+BiasAdd +activation epilogue)
* :func:`dense`          -- ``tf.layers.dense`` forward/backward (autograd)
* :func:`softmax_xent`   -- ``tf.nn.softmax_cross_entropy_with_logits`` +
                            ``reduce_mean`` + accuracy (autograd)
"""
from __future__ import annotations

import torch

from ._ext import check_gpu_f32, hip, ptr, stream_handle

ACT = {None: 0, "none": 0, "linear": 0, "sigmoid": 1, "relu": 2, "gelu": 3}


def _act_id(act):
    if isinstance(act, int):
        return act
    try:
        return ACT[act]
    except KeyError:
        raise ValueError("unknown activation %r" % (act,))


def _aligned(t):
    return t if (t.data_ptr() % 16 == 0 and t.is_contiguous()) else t.contiguous().clone()


# ---------------------------------------------------------------------------
# CPU reference math
# ---------------------------------------------------------------------------
def _act_ref(x, act):
    if act == 1:
        return torch.sigmoid(x)
    if act == 2:
        return torch.relu(x)
    if act == 3:
        return torch.nn.functional.gelu(x, approximate="tanh")
    return x


def _act_grad_ref(dy, s, act):
    if act == 1:
        return dy * s * (1 - s)
    if act == 2:
        return dy * (s > 0).to(dy.dtype)
    if act == 3:
        k0, k1 = 0.7978845608028654, 0.044715
        th = torch.tanh(k0 * (s + k1 * s ** 3))
        return dy * (0.5 * (1 + th) + 0.5 * s * (1 - th * th) * k0 * (1 + 3 * k1 * s * s))
    return dy


# ---------------------------------------------------------------------------
# GEMM
# ---------------------------------------------------------------------------
def gemm(a, b, trans_a=False, trans_b=False, bias=None, act=None, aux=None, act_grad=False,
         alpha=1.0, beta=0.0, out=None):
    """``out = epi(alpha * op(a) @ op(b))`` with fused bias/activation.

    ``act_grad=True`` multiplies by ``act'(aux)`` instead of applying ``act``
    (aux = saved forward output for sigmoid/relu, pre-activation for gelu).
    """
    act = _act_id(act)
    M = a.shape[1] if trans_a else a.shape[0]
    K = a.shape[0] if trans_a else a.shape[1]
    Kb = b.shape[1] if trans_b else b.shape[0]
    N = b.shape[0] if trans_b else b.shape[1]
    if K != Kb:
        raise ValueError("gemm: inner dims differ (%d vs %d)" % (K, Kb))
    if not a.is_cuda:
        A = a.t() if trans_a else a
        B = b.t() if trans_b else b
        y = alpha * (A @ B)
        if act_grad:
            y = _act_grad_ref(y, aux, act)
        else:
            if bias is not None:
                y = y + bias
            y = _act_ref(y, act)
        if out is not None:
            if beta != 0.0:
                y = y + beta * out
            out.copy_(y)
            return out
        return y
    check_gpu_f32(a, b, bias, aux, out)
    if out is None:
        if beta != 0.0:
            raise ValueError("gemm: beta != 0 needs out")
        out = torch.empty((M, N), device=a.device, dtype=torch.float32)
    check_gpu_f32(out)
    if tuple(out.shape) != (M, N):
        raise ValueError("gemm: out has shape %s, expected %s" % (tuple(out.shape), (M, N)))
    if act_grad and (aux is None or tuple(aux.shape) != (M, N)):
        raise ValueError("gemm: act_grad needs aux of shape (M, N)")
    if bias is not None and bias.numel() != N:
        raise ValueError("gemm: bias must have N elements")
    hip().gemm_f32(trans_a, trans_b, M, N, K, float(alpha), ptr(a), a.stride(0), ptr(b),
                   b.stride(0), float(beta), ptr(out), out.stride(0), ptr(bias), act, ptr(aux),
                   aux.stride(0) if aux is not None else 0, bool(act_grad), stream_handle())
    return out


def colsum(g, out=None, beta=0.0):
    """Column sums of a 2-D tensor (BiasAddGrad)."""
    if not g.is_cuda:
        s = g.sum(0)
        if out is None:
            return s
        out.copy_(s + beta * out if beta else s)
        return out
    check_gpu_f32(g, out)
    M, N = g.shape
    if out is None:
        out = torch.empty(N, device=g.device, dtype=torch.float32)
    hip().colsum(M, N, ptr(g), g.stride(0), float(beta), ptr(out), stream_handle())
    return out


def act_backward(dy, s, act):
    act = _act_id(act)
    if not dy.is_cuda:
        return _act_grad_ref(dy, s, act)
    dy = _aligned(dy)
    s = _aligned(s)
    check_gpu_f32(dy, s)
    dz = torch.empty_like(dy)
    hip().act_bwd(dy.numel(), act, ptr(dy), ptr(s), ptr(dz), stream_handle())
    return dz


def activation(x, act):
    act = _act_id(act)
    if not x.is_cuda:
        return _act_ref(x, act)
    x = _aligned(x)
    check_gpu_f32(x)
    y = torch.empty_like(x)
    hip().act_fwd(x.numel(), act, ptr(x), ptr(y), stream_handle())
    return y


# ---------------------------------------------------------------------------
# dense layer (tf.layers.dense): y = act(x @ W^T + b), W stored [out, in]
# ---------------------------------------------------------------------------
class _DenseFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act):
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        y = gemm(x2, w, trans_b=True, bias=b, act=act)
        # GELU's derivative needs the pre-activation; sigmoid/relu use the output.
        if act == 3:
            z = gemm(x2, w, trans_b=True, bias=b, act=0)
            ctx.save_for_backward(x2, w, z)
        else:
            ctx.save_for_backward(x2, w, y)
        ctx.act = act
        ctx.has_bias = b is not None
        ctx.xshape = x.shape
        return y.reshape(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w, s = ctx.saved_tensors
        dy2 = dy.reshape(-1, w.shape[0]).contiguous()
        dz = act_backward(dy2, s, ctx.act) if ctx.act else dy2
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = gemm(dz, w).reshape(ctx.xshape)          # dz @ W     [M, in]
        if ctx.needs_input_grad[1]:
            dw = gemm(dz, x2, trans_a=True)                # dz^T @ x   [out, in]
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = colsum(dz)
        return dx, dw, db, None


def dense(x, w, b=None, act=None):
    return _DenseFn.apply(x, w, b, _act_id(act))


# ---------------------------------------------------------------------------
# softmax cross-entropy (+ mean over rows, + accuracy)
# ---------------------------------------------------------------------------
def softmax_xent_stats(logits, labels, ignore_index=-100, want_grad=True, scale=None):
    """Returns (loss_rows, dlogits or None, correct_rows).

    ``labels``: int class ids [N] or dense/one-hot float [N, C] (TF semantics).
    dlogits is pre-scaled by ``scale`` (default 1/N, the reduce_mean).
    """
    N, C = logits.shape
    dense_lab = labels.dtype.is_floating_point
    if scale is None:
        scale = 1.0 / max(N, 1)
    if not logits.is_cuda:
        lse = torch.logsumexp(logits, dim=1)
        p = torch.softmax(logits, dim=1)
        am = logits.argmax(dim=1)
        if dense_lab:
            loss = (labels * (lse[:, None] - logits)).sum(1)
            correct = (am == labels.argmax(dim=1)).float()
            d = (p * labels.sum(1, keepdim=True) - labels) * scale if want_grad else None
        else:
            lab = labels.long()
            valid = (lab != ignore_index) & (lab >= 0) & (lab < C)
            safe = torch.where(valid, lab, torch.zeros_like(lab))
            loss = torch.where(valid, lse - logits.gather(1, safe[:, None])[:, 0],
                               torch.zeros_like(lse))
            correct = ((am == lab) & valid).float()
            if want_grad:
                oh = torch.nn.functional.one_hot(safe, C).to(logits.dtype)
                d = (p - oh) * valid[:, None].to(logits.dtype) * scale
            else:
                d = None
        return loss, d, correct
    logits = logits.contiguous()
    check_gpu_f32(logits)
    loss = torch.empty(N, device=logits.device, dtype=torch.float32)
    correct = torch.empty(N, device=logits.device, dtype=torch.float32)
    d = torch.empty_like(logits) if want_grad else None
    if dense_lab:
        lab = labels.contiguous().float()
        hip().softmax_xent(N, C, ptr(logits), C, 0, ptr(lab), C, -1, float(scale), ptr(loss),
                           ptr(d), C, ptr(correct), 0, stream_handle())
    else:
        lab = labels.to(torch.int32).contiguous()
        hip().softmax_xent(N, C, ptr(logits), C, ptr(lab), 0, 0, int(ignore_index), float(scale),
                           ptr(loss), ptr(d), C, ptr(correct), 0, stream_handle())
    return loss, d, correct


class _SoftmaxXentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index):
        loss_rows, d, correct = softmax_xent_stats(logits, labels, ignore_index, True)
        ctx.save_for_backward(d)
        ctx.mark_non_differentiable(correct)
        return loss_rows.mean(), correct.mean()

    @staticmethod
    def backward(ctx, dloss, dacc):
        (d,) = ctx.saved_tensors
        return d * dloss, None, None


def softmax_cross_entropy(logits, labels, ignore_index=-100):
    """(mean loss, accuracy) -- worker.py:63-66 and 87-90 in one fused kernel."""
    return _SoftmaxXentFn.apply(logits, labels, ignore_index)
