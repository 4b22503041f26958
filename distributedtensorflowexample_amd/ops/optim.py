"""Flat multi-tensor optimizer kernels (one launch per optimizer step).

Parameters of a model live in ONE flat f32 buffer (``models.flat``), so the
SGD of ``GradientDescentOptimizer`` (worker.py:71, ``ApplyGradientDescent`` x4
on the ps, worker.py:79) is a single dwordx4 kernel over 79,510 elements.
"""
from __future__ import annotations

import torch

from ._ext import check_gpu_f32, hip, ptr, stream_handle


def sgd_(p, g, lr, weight_decay=0.0, lr_tensor=None):
    if not p.is_cuda:
        with torch.no_grad():
            if weight_decay:
                p.add_(p, alpha=-float(lr) * weight_decay)
            p.add_(g, alpha=-float(lr if lr_tensor is None else lr_tensor.item()))
        return p
    check_gpu_f32(p, g, lr_tensor)
    hip().sgd(p.numel(), ptr(p), ptr(g), float(lr), ptr(lr_tensor), float(weight_decay),
              stream_handle())
    return p


def momentum_(p, g, buf, lr, momentum=0.9, weight_decay=0.0, nesterov=False, lr_tensor=None):
    if not p.is_cuda:
        with torch.no_grad():
            l = float(lr if lr_tensor is None else lr_tensor.item())
            gg = g + weight_decay * p
            buf.mul_(momentum).add_(gg)
            p.add_(gg + momentum * buf if nesterov else buf, alpha=-l)
        return p
    check_gpu_f32(p, g, buf, lr_tensor)
    hip().momentum(p.numel(), ptr(p), ptr(g), ptr(buf), float(lr), ptr(lr_tensor),
                   float(momentum), float(weight_decay), bool(nesterov), stream_handle())
    return p


def adam_(p, g, m, v, lr, step, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0,
          adamw=True, lr_tensor=None, step_tensor=None):
    """Bias-corrected Adam/AdamW.  ``step`` is 1-based (after increment)."""
    if not p.is_cuda:
        with torch.no_grad():
            l = float(lr if lr_tensor is None else lr_tensor.item())
            t = int(step if step_tensor is None else step_tensor.item())
            gg = g if adamw else g + weight_decay * p
            m.mul_(beta1).add_(gg, alpha=1 - beta1)
            v.mul_(beta2).addcmul_(gg, gg, value=1 - beta2)
            bc1 = 1 - beta1 ** t
            bc2 = 1 - beta2 ** t
            denom = v.sqrt() / (bc2 ** 0.5) + eps
            if adamw:
                p.mul_(1 - l * weight_decay)
            p.addcdiv_(m, denom, value=-l / bc1)
        return p
    check_gpu_f32(p, g, m, v, lr_tensor)
    if step_tensor is not None and step_tensor.dtype != torch.int32:
        raise TypeError("step_tensor must be int32")
    hip().adam(p.numel(), ptr(p), ptr(g), ptr(m), ptr(v), float(lr), ptr(lr_tensor),
               float(beta1), float(beta2), float(eps), float(weight_decay), bool(adamw),
               int(step), ptr(step_tensor), stream_handle())
    return p


def scale_(x, a):
    if not x.is_cuda:
        x.mul_(a)
        return x
    check_gpu_f32(x)
    hip().scale(x.numel(), ptr(x), float(a), stream_handle())
    return x


def counter_add_(c, d=1):
    """In-place device add on an int32 scalar counter (capture-safe)."""
    if not c.is_cuda:
        c.add_(d)
        return c
    if c.dtype != torch.int32:
        raise TypeError("counter must be int32")
    hip().counter_add(ptr(c), int(d), stream_handle())
    return c
