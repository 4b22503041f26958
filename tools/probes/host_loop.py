"""Short timed regions (bench.py --steps 20 --warmup 5): graph replay vs the C++ host loop
(``FusedMLPTrainer.run_launched``) vs a hybrid (a few host-launched steps, then the graph),
interleaved rounds in one process; plus numerics: all three give the same parameters."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributedtensorflowexample_amd.data.synthetic import mnist_like_device  # noqa: E402
from distributedtensorflowexample_amd.models.mlp import init_params  # noqa: E402
from distributedtensorflowexample_amd.train.fused_mlp import FusedMLPTrainer  # noqa: E402


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e6


def main():
    dev = torch.device("cuda:0")
    x, y = mnist_like_device(55000, seed=100, device=dev)
    p0 = init_params(dev, seed=1234)
    out = {}
    # numerics: 37 steps three ways from the same start
    finals = {}
    for mode in ("graph", "host", "hybrid"):
        tr = FusedMLPTrainer(p0, x, y)
        tr.run(5)
        if mode == "graph":
            tr.run(32)
        elif mode == "host":
            tr.run_launched(32)
        else:
            tr.prepare(32, lead=4)
            tr.run(32, lead=4)
        finals[mode] = tr.flush().clone()
    out["host_vs_graph_maxdiff"] = float((finals["host"] - finals["graph"]).abs().max())
    out["hybrid_vs_graph_maxdiff"] = float((finals["hybrid"] - finals["graph"]).abs().max())
    for K in (20, 200, 2000):
        res = {"graph": [], "host": [], "hybrid2": [], "hybrid4": []}
        tr = FusedMLPTrainer(p0, x, y)
        tr.run(5)
        for _ in range(5):
            for mode in res:
                lead = {"graph": 0, "host": 0, "hybrid2": 2, "hybrid4": 4}[mode]
                if mode != "host":
                    tr.prepare(K, lead=lead)
                    t = timed(lambda: (tr.run(K, lead=lead), tr.flush()))
                else:
                    t = timed(lambda: (tr.run_launched(K), tr.flush()))
                res[mode].append(t / K)
                tr.run(1, use_graph=False)
        out["K%d_us_per_step" % K] = {m: [round(min(v), 3), round(sorted(v)[len(v) // 2], 3)]
                                      for m, v in res.items()}
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
