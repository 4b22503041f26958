"""Where do the fixed costs of a SHORT timed region go (bench.py --steps 20 --warmup 5)?

Times, on one GPU: an empty synchronize round trip; the first and the second replay of a
freshly captured 20-step graph; flush() alone; 20 eager steps; the full bench sequence.
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributedtensorflowexample_amd.data.synthetic import mnist_like_device  # noqa: E402
from distributedtensorflowexample_amd.models.mlp import init_params  # noqa: E402
from distributedtensorflowexample_amd.train.fused_mlp import FusedMLPTrainer  # noqa: E402


def t_us(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e6


def main():
    dev = torch.device("cuda:0")
    K = int(os.environ.get("K", "20"))
    res = {}
    x, y = mnist_like_device(55000, seed=100, device=dev)
    tr = FusedMLPTrainer(init_params(dev, seed=1234), x, y)
    res["sync_only"] = min(t_us(lambda: None) for _ in range(20))
    tr.run(5)
    for rep in range(3):  # the bench sequence, fresh graph each time
        tr.prepare(K)
        res["bench_seq_%d" % rep] = t_us(lambda: (tr.run(K), tr.flush()))
        tr.run(1, use_graph=False)
    for rep in range(3):
        tr.prepare(K)
        res["run_only_first_replay_%d" % rep] = t_us(lambda: tr.run(K))
        res["flush_only_%d" % rep] = t_us(lambda: tr.flush())
        tr.run(1, use_graph=False)
    # same graph replayed twice (state is not meaningful, timing is)
    g = tr._graph(K)
    res["replay_a"] = t_us(g.replay)
    res["replay_b"] = t_us(g.replay)
    res["replay_c"] = t_us(g.replay)
    res["eager_%d" % K] = min(t_us(lambda: tr.run(K, use_graph=False)) for _ in range(3))
    res["eager_1"] = min(t_us(lambda: tr.run(1, use_graph=False)) for _ in range(5))
    print(json.dumps({k: round(v, 2) for k, v in res.items()}, indent=1), flush=True)


if __name__ == "__main__":
    main()
