"""Synthetic MNIST-shaped data (the train images are absent from the reference,
.MISSING_LARGE_BLOBS:1, and there is no network to fetch them).

``mnist_like`` draws 10 class prototypes in [0, 1]^784 and samples noisy,
clipped copies, so the data has the reference's shapes/ranges (x f32 in
[0, 1] shaped [N, 784], labels 0..9) AND is learnable -- loss curves and
accuracy behave like MNIST training rather than fitting noise.
"""
from __future__ import annotations

import torch


def mnist_like(n, seed=0, device="cpu", noise=0.35, sparsity=0.55):
    g = torch.Generator().manual_seed(int(seed))
    proto = torch.rand(10, 784, generator=g)
    proto = proto * (torch.rand(10, 784, generator=g) > sparsity)
    y = torch.randint(0, 10, (n,), generator=g)
    x = (proto[y] + noise * torch.randn(n, 784, generator=g)).clamp_(0.0, 1.0)
    return x.to(device), y.to(torch.int32).to(device)


def mnist_like_device(n, seed, device, noise=0.35, sparsity=0.55):
    """Same distribution generated directly in HBM (no host->device copy of N rows)."""
    g = torch.Generator(device=device).manual_seed(int(seed))
    proto = torch.rand(10, 784, generator=g, device=device)
    proto = proto * (torch.rand(10, 784, generator=g, device=device) > sparsity)
    y = torch.randint(0, 10, (n,), generator=g, device=device)
    x = (proto[y] + noise * torch.randn(n, 784, generator=g, device=device)).clamp_(0.0, 1.0)
    return x, y.to(torch.int32)
