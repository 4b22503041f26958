"""Standalone timing of the bf16 column sum (bias gradient) at BERT's decoder shape.

    python tools/probes/colsum_one.py [rows] [cols]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributedtensorflowexample_amd.ops import bf16 as B16  # noqa: E402


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 2432
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 30528
    dev = torch.device("cuda:0")
    g = (torch.randn(M, N, device=dev) * 0.1).to(torch.bfloat16)
    out = torch.zeros(N, device=dev)
    ref = g.float().sum(0)
    B16.colsum(g, out=out, beta=0.0)
    err = (out - ref).abs().max().item()
    ts = []
    for _ in range(7):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            B16.colsum(g, out=out, beta=1.0)
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / 20 * 1e3)
    ts.sort()
    print(json.dumps({"M": M, "N": N, "us": round(ts[3], 2), "range": [round(ts[0], 2), round(ts[-1], 2)],
                      "TBps": round(M * N * 2 / ts[3] / 1e6, 2), "max_err": err}))


if __name__ == "__main__":
    main()
