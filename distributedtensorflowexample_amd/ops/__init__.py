"""Compute ops: hand-written gfx950 HIP kernels behind thin Python wrappers."""
from ._ext import hip, hip_available, host
from . import init, mlp_step, nn, optim
from .nn import activation, colsum, dense, gemm, softmax_cross_entropy, softmax_xent_stats

__all__ = [
    "hip", "hip_available", "host", "init", "mlp_step", "nn", "optim", "activation", "colsum",
    "dense", "gemm", "softmax_cross_entropy", "softmax_xent_stats",
]
