"""Split-K / tile sweep of the BERT-base weight-gradient GEMMs (f32 accumulate path).

    DTFX_GEMM_CFG=<0..3> python tools/gemm_sweep.py     (the tile is read once per process)

One JSON line per (shape, splitk): microseconds and TFLOP/s of dW += dY^T . X.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedtensorflowexample_amd.ops import bf16  # noqa: E402
from tools.gemm_bench import timeit  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    T = 128 * 128
    shapes = [("ffn_in_wgrad", 3072, 768, T), ("ffn_out_wgrad", 768, 3072, T),
              ("qkv_wgrad", 2304, 768, T), ("attn_out_wgrad", 768, 768, T)]
    cfg = os.environ.get("DTFX_GEMM_CFG", "auto")
    for name, M, N, K in shapes:
        a = torch.randn(K, M, device=dev).to(torch.bfloat16)
        b = torch.randn(K, N, device=dev).to(torch.bfloat16)
        out = torch.zeros(M, N, device=dev, dtype=torch.float32)
        ref = a.float().t() @ b.float()
        for sk in (0, 1, 2, 3, 4, 6, 8, 12, 16):
            try:
                t = timeit(lambda: bf16.gemm(a, b, True, False, out=out, beta=1.0, splitk=sk))
                out.zero_()
                bf16.gemm(a, b, True, False, out=out, beta=1.0, splitk=sk)
                err = float((out - ref).abs().max())
            except Exception as e:  # unsupported combination
                print(json.dumps({"shape": name, "cfg": cfg, "splitk": sk, "error": str(e)[:80]}))
                continue
            print(json.dumps({"shape": name, "cfg": cfg, "splitk": sk, "us": round(t * 1e6, 1),
                              "tflops": round(2.0 * M * N * K / t / 1e12, 1),
                              "max_abs_err": err}), flush=True)


if __name__ == "__main__":
    main()
