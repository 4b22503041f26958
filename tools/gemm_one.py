"""Run one bf16 GEMM shape a few times (for rocprofv3 counter collection)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedtensorflowexample_amd.ops import bf16  # noqa: E402

M, N, K = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (8192, 8192, 8192)))
ta, tb = (sys.argv[4] == "1", sys.argv[5] == "1") if len(sys.argv) > 5 else (False, True)
dev = torch.device("cuda:0")
a = torch.randn(*((K, M) if ta else (M, K)), device=dev).to(torch.bfloat16)
b = torch.randn(*((N, K) if tb else (K, N)), device=dev).to(torch.bfloat16)
# weight gradients (A^T) accumulate into f32 gradient buffers, as in training (split-K path)
out = torch.zeros(M, N, device=dev, dtype=torch.float32 if ta else torch.bfloat16)
for _ in range(5):
    bf16.gemm(a, b, ta, tb, out=out, beta=1.0 if ta else 0.0)
torch.cuda.synchronize()
print("done", M, N, K, ta, tb)
