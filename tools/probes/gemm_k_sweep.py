"""Per-tile fixed cost of the 8-phase bf16 GEMM: time(K) at fixed M x N, plain bf16 output, fitted
as a + b*K.  The intercept is the K-independent part per launch (prologue pipeline fill,
epilogue, launch / drain) -- what a persistent multi-tile block could overlap.

    python tools/probes/gemm_k_sweep.py [--cfg 5]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributedtensorflowexample_amd.ops import bf16  # noqa: E402
from distributedtensorflowexample_amd.ops._ext import hip  # noqa: E402


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    hip().gemm_bf16_set_cfg(a.cfg)
    for M, N in ((16384, 3072), (16384, 768), (8192, 8192)):
        ks = (768, 1536, 3072, 6144)
        ts = []
        for K in ks:
            x = (torch.rand(M, K, device=dev) - 0.5).to(torch.bfloat16)
            w = (torch.rand(N, K, device=dev) - 0.5).to(torch.bfloat16)
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            r = sorted(timeit(lambda: bf16.gemm(x, w, False, True, out=out)) for _ in range(a.rounds))
            ts.append(r[len(r) // 2])
        n = len(ks)
        mk, mt = sum(ks) / n, sum(ts) / n
        b = sum((k - mk) * (t - mt) for k, t in zip(ks, ts)) / sum((k - mk) ** 2 for k in ks)
        icpt = mt - b * mk
        print(json.dumps({"M": M, "N": N, "cfg": a.cfg, "K": list(ks), "us": [round(t, 2) for t in ts],
                          "tflops": [round(2.0 * M * N * k / t / 1e6, 1) for k, t in zip(ks, ts)],
                          "intercept_us": round(icpt, 2), "us_per_k64": round(b * 64, 3)}), flush=True)
    hip().gemm_bf16_set_cfg(-1)


if __name__ == "__main__":
    main()
