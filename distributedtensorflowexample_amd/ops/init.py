"""Parameter initializers (``tf.random_normal_initializer`` et al.).

GPU tensors are filled by the Philox4x32-10 HIP kernel (counter-based, so a
(seed, offset) pair reproduces the same values on every rank -- sync-DP
replicas start bit-identical without a broadcast).  CPU tensors use a
torch.Generator with the same seed (different stream of numbers, same
distribution).
"""
from __future__ import annotations

import torch

from ._ext import check_gpu_f32, hip, ptr, stream_handle

_MODES = {"normal": 0, "uniform": 1, "truncated_normal": 2}


def fill_(t, kind="normal", a=0.0, b=1.0, seed=0, offset=0):
    """normal: mean=a std=b; uniform: [a, b); truncated_normal: mean a, std b, |z|<=2."""
    mode = _MODES[kind]
    if not t.is_cuda:
        gen = torch.Generator().manual_seed((int(seed) * 1000003 + int(offset)) & 0x7FFFFFFFFFFFFFFF)
        with torch.no_grad():
            if mode == 0:
                t.copy_(torch.randn(t.shape, generator=gen) * b + a)
            elif mode == 1:
                t.copy_(torch.rand(t.shape, generator=gen) * (b - a) + a)
            else:
                z = torch.randn(t.shape, generator=gen)
                for _ in range(16):
                    bad = z.abs() > 2
                    if not bad.any():
                        break
                    z = torch.where(bad, torch.randn(t.shape, generator=gen), z)
                t.copy_(z.clamp(-2, 2) * b + a)
        return t
    check_gpu_f32(t)
    hip().philox_init(t.numel(), ptr(t), int(seed) & 0xFFFFFFFFFFFFFFFF,
                      int(offset) & 0xFFFFFFFFFFFFFFFF, mode, float(a), float(b), stream_handle())
    return t
