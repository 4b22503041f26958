"""bf16 GEMM throughput: hand-written MFMA kernel vs torch.matmul (hipBLASLt).

Shapes are the BERT-base training GEMMs (tokens = batch x seq) and a large
square; prints one JSON line per shape with TFLOP/s of both.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedtensorflowexample_amd.ops import bf16  # noqa: E402


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    dev = torch.device("cuda:0")
    T = 32 * 512
    shapes = [  # (name, M, N, K, ta, tb)
        ("qkv_fwd", T, 2304, 768, False, True), ("ffn1_fwd", T, 3072, 768, False, True),
        ("ffn2_fwd", T, 768, 3072, False, True), ("ffn1_dgrad", T, 768, 3072, False, False),
        ("ffn1_wgrad", 3072, 768, T, True, False), ("sq4096", 4096, 4096, 4096, False, True),
        ("sq8192", 8192, 8192, 8192, False, True)]
    for name, M, N, K, ta, tb in shapes:
        a = torch.randn(*((K, M) if ta else (M, K)), device=dev).to(torch.bfloat16)
        b = torch.randn(*((N, K) if tb else (K, N)), device=dev).to(torch.bfloat16)
        A = a.t() if ta else a
        B = b.t() if tb else b
        if ta:  # weight gradients accumulate into f32 master-gradient buffers (split-K path)
            out = torch.zeros(M, N, device=dev, dtype=torch.float32)
            t_ours = timeit(lambda: bf16.gemm(a, b, ta, tb, out=out, beta=1.0))
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        else:
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            t_ours = timeit(lambda: bf16.gemm(a, b, ta, tb, out=out))
        t_lib = timeit(lambda: torch.matmul(A, B, out=out))
        fl = 2.0 * M * N * K
        err = (bf16.gemm(a, b, ta, tb, out_dtype=torch.float32) - A.float() @ B.float()).abs().max()
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "ours_tflops": round(fl / t_ours / 1e12, 1),
                          "hipblaslt_tflops": round(fl / t_lib / 1e12, 1),
                          "ours_us": round(t_ours * 1e6, 1), "max_abs_err": float(err)}), flush=True)


if __name__ == "__main__":
    main()
