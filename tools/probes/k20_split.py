"""Fixed cost of a short MLP timed region, split (round 6): bench.py's host-loop region
(``run_launched(K, flush=True)`` between two ``torch.cuda.synchronize()``) timed at several K,
interleaved, medians over many repetitions -> t(K) = a + b K; the host time of the launching
call itself; the flush's share (the same K with and without the flush launch); the completion
wait (device synchronize vs a stream synchronize vs an event).

    python tools/probes/k20_split.py [--reps 41]

One JSON line.
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


def med(v):
    v = sorted(v)
    return v[len(v) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=41)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    x, y = mnist_like_device(55000, seed=100, device=dev)
    tr = FusedMLPTrainer(init_params(dev, seed=1234), x, y)
    tr.run(5)
    tr.run_launched(50, flush=True)
    tr.run(1, use_graph=False)
    Ks = (1, 5, 10, 20, 40)
    region = {k: [] for k in Ks}
    noflush = {k: [] for k in Ks}
    call = {k: [] for k in Ks}
    waits = {"device": [], "stream": [], "event": [], "stream+device": []}
    s = torch.cuda.current_stream()
    for _ in range(a.reps):
        for k in Ks:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tr.run_launched(k, flush=True)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            region[k].append((t2 - t0) * 1e6)
            call[k].append((t1 - t0) * 1e6)
            tr.run(1, use_graph=False)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tr.run_launched(k, flush=False)
            torch.cuda.synchronize()
            noflush[k].append((time.perf_counter() - t0) * 1e6)
        for how in waits:
            ev = torch.cuda.Event()
            tr.run(1, use_graph=False)  # the same preamble as bench.py's timed region
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tr.run_launched(20, flush=True)
            if how == "device":
                torch.cuda.synchronize()
            elif how == "stream":
                s.synchronize()
            elif how == "stream+device":
                s.synchronize()
                torch.cuda.synchronize()
            else:
                ev.record(s)
                ev.synchronize()
            waits[how].append((time.perf_counter() - t0) * 1e6)
    out = {"region_us": {k: round(med(v), 2) for k, v in region.items()},
           "region_noflush_us": {k: round(med(v), 2) for k, v in noflush.items()},
           "host_call_us": {k: round(med(v), 2) for k, v in call.items()},
           "k20_wait_us": {k: round(med(v), 2) for k, v in waits.items()}}
    r = out["region_us"]
    b = (r[40] - r[10]) / 30.0
    out["fit_us"] = {"per_step": round(b, 3), "fixed": round(r[20] - 20 * b, 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
