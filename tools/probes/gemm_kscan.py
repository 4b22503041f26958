"""Fixed (per-tile prologue + epilogue) vs per-K-tile cost of the bf16 GEMM: time
M x N x K for several K at fixed M, N (ours, auto config, and hipBLASLt via torch.matmul),
fit t = a + b * K.  One JSON line per (shape, epilogue, K) and one fit line per series.

    python tools/probes/gemm_kscan.py [--M 16384 --N 3072 --Ks 768,1536,3072,6144]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributedtensorflowexample_amd.ops import bf16, hip  # noqa: E402


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(3):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / iters * 1e3)
    return best  # us


def fit(ks, ts):
    n = len(ks)
    mk, mt = sum(ks) / n, sum(ts) / n
    b = sum((k - mk) * (t - mt) for k, t in zip(ks, ts)) / sum((k - mk) ** 2 for k in ks)
    return mt - b * mk, b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=16384)
    ap.add_argument("--N", type=int, default=3072)
    ap.add_argument("--Ks", default="768,1536,3072,6144")
    ap.add_argument("--epis", default="plain,gelu")
    ap.add_argument("--cfgs", default="", help="comma list of forced tile configs (plain epilogue)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    M, N = a.M, a.N
    Ks = [int(k) for k in a.Ks.split(",")]
    series = {}
    for K in Ks:
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        bias = torch.zeros(N, device=dev)
        runs = {"hipblaslt": lambda: torch.matmul(x, w.t())}
        if "plain" in a.epis:
            runs["plain"] = lambda: bf16.gemm(x, w, False, True, out=out)
        if "gelu" in a.epis:
            runs["gelu"] = lambda: bf16.gemm(x, w, False, True, bias=bias, act="gelu", aux_out=aux, out=out)
        for c in [int(v) for v in a.cfgs.split(",") if v]:
            def run_cfg(c=c):
                hip().gemm_bf16_set_cfg(c)
                bf16.gemm(x, w, False, True, out=out)
                hip().gemm_bf16_set_cfg(-1)
            runs["cfg%d" % c] = run_cfg
        for name, fn in runs.items():
            us = timeit(fn)
            tf = 2.0 * M * N * K / us * 1e-6
            series.setdefault(name, []).append((K, us))
            print(json.dumps({"M": M, "N": N, "K": K, "kind": name, "us": round(us, 2),
                              "tflops": round(tf, 1)}), flush=True)
    for name, pts in series.items():
        a0, b0 = fit([p[0] for p in pts], [p[1] for p in pts])
        print(json.dumps({"fit": name, "M": M, "N": N, "fixed_us": round(a0, 2),
                          "us_per_k64": round(b0 * 64, 3)}), flush=True)


if __name__ == "__main__":
    main()
