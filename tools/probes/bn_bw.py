"""BatchNorm elementwise kernels at ResNet-50's largest activation (256 x 56 x 56 x 256 bf16):
achieved HBM bandwidth of bn_apply (+ReLU, +/- residual) and bn_bwd_apply, one JSON line each."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from distributedtensorflowexample_amd.ops import cnn  # noqa: E402
from tools.gemm_bench import timeit  # noqa: E402

dev = torch.device("cuda:0")
N, H, W, C = 256, 56, 56, 256
x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
r = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
de = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
mean, rstd = torch.zeros(C, device=dev), torch.ones(C, device=dev)
g, b = torch.ones(C, device=dev), torch.zeros(C, device=dev)
sdy, sdx = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
n = x.numel()
for name, nbytes, fn in [
    ("bn_apply_relu", 4 * n, lambda: cnn.bn_apply(x, mean, rstd, g, b, None, relu=True)),
    ("bn_apply_res_relu", 6 * n, lambda: cnn.bn_apply(x, mean, rstd, g, b, r, relu=True)),
    ("bn_bwd_apply", 6 * n, lambda: cnn.bn_bwd_apply(de, x, mean, rstd, g, sdy, sdx)),
    ("copy_bf16 (torch)", 4 * n, lambda: r.copy_(x)),
]:
    t = timeit(fn, iters=20)
    print(json.dumps({"kernel": name, "us": round(t * 1e6, 1), "TBps": round(nbytes / t / 1e12, 2)}))
