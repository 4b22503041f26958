"""bf16 column sums at the MLM decoder bias-gradient shape (2432 x 30522, ld 30528): 4 vs 8 rows
in flight per thread (DTFX_COLSUM_U), interleaved; us per call and the read rate.  One JSON line.

    python tools/probes/colsum_u.py [--rows 2432 --cols 30522 --iters 200 --rounds 5]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from distributedtensorflowexample_amd.ops import bf16, hip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2432)
    ap.add_argument("--cols", type=int, default=30522)
    ap.add_argument("--ld", type=int, default=30528)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.randn(a.rows, a.ld, device=dev).to(torch.bfloat16)[:, :a.cols]
    out = torch.zeros(a.cols, device=dev)
    res = {4: [], 8: []}
    try:
        for _ in range(a.rounds):
            for u in (4, 8):
                hip().colsum_set_rows_in_flight(u)
                for _ in range(5):
                    bf16.colsum(g, out=out)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    bf16.colsum(g, out=out)
                e1.record()
                torch.cuda.synchronize()
                res[u].append(e0.elapsed_time(e1) * 1e3 / a.iters)
    finally:
        hip().colsum_set_rows_in_flight(0)
    line = {"rows": a.rows, "cols": a.cols, "ld": a.ld, "iters": a.iters}
    for u, v in res.items():
        med = sorted(v)[len(v) // 2]
        line["u%d" % u] = {"us_median": round(med, 2), "all": [round(t, 2) for t in v],
                           "TB_per_s": round(a.rows * a.ld * 2 / med / 1e6, 2)}
    print(json.dumps(line))


if __name__ == "__main__":
    main()
