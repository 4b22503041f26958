"""Where the flush launch's cost in a short MLP region comes from (round 6).

Interleaved variants with the SAME preamble (one eager step + synchronize), medians over reps:
  flush     run_launched(K, flush=True)                       -- bench.py's timed region
  noflush   run_launched(K, flush=False)                      (the update left pending)
  plus1     run_launched(K + 1, flush=False)                  (one more step instead of a flush)
  sep       run_launched(K, flush=False); flush() in Python   (the flush as its own call)
Every variant's pending update is applied after its clock (untimed), so all start alike.

    python tools/probes/k20_flush.py [--reps 41] [--K 20]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributedtensorflowexample_amd.data.synthetic import mnist_like_device  # noqa: E402
from distributedtensorflowexample_amd.models.mlp import init_params  # noqa: E402
from distributedtensorflowexample_amd.train.fused_mlp import FusedMLPTrainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=41)
    ap.add_argument("--K", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    x, y = mnist_like_device(55000, seed=100, device=dev)
    tr = FusedMLPTrainer(init_params(dev, seed=1234), x, y)
    tr.run(5)
    tr.run_launched(50, flush=True)
    K = a.K
    res = {v: [] for v in ("flush", "noflush", "plus1", "sep")}
    for _ in range(a.reps):
        for v in res:
            tr.run(1, use_graph=False)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if v == "flush":
                tr.run_launched(K, flush=True)
            elif v == "noflush":
                tr.run_launched(K, flush=False)
            elif v == "plus1":
                tr.run_launched(K + 1, flush=False)
            else:
                tr.run_launched(K, flush=False)
                tr.flush()
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t0) * 1e6)
            tr.flush()
    med = {v: round(sorted(t)[len(t) // 2], 2) for v, t in res.items()}
    print(json.dumps({"K": K, "reps": a.reps, "region_us": med,
                      "flush_cost_us": round(med["flush"] - med["noflush"], 2),
                      "step_cost_us": round(med["plus1"] - med["noflush"], 2)}), flush=True)


if __name__ == "__main__":
    main()
