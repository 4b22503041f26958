"""Fixed vs per-step cost of a replayed MLP-step hipGraph: t(n) = a + b * n.

Replays graphs of n steps (state irrelevant: timing only), after an idle gap and
back-to-back, to separate the graph-launch cost from the per-step cost and
from clock ramp-up after idle.
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
    x, y = mnist_like_device(55000, seed=100, device=dev)
    tr = FusedMLPTrainer(init_params(dev, seed=1234), x, y)
    tr.run(5)
    res = {"env": {k: v for k, v in os.environ.items() if k.startswith(("DEBUG_", "HIP_", "GPU_"))}}
    busy = torch.empty(64 << 20, device=dev)
    for n in (1, 2, 5, 10, 20, 50, 100, 400):
        g = tr._graph(n)
        g.replay()
        torch.cuda.synchronize()
        time.sleep(0.05)
        idle = t_us(g.replay)
        b2b = min(t_us(g.replay) for _ in range(5))
        # GPU kept busy right up to the launch (clocks up), then the graph
        def hot():
            busy.mul_(1.0)
            g.replay()
        hot_t = min(t_us(hot) for _ in range(3)) - min(t_us(lambda: busy.mul_(1.0)) for _ in range(3))
        res[n] = {"after_idle": round(idle, 2), "back_to_back": round(b2b, 2),
                  "after_busy_kernel": round(hot_t, 2)}
    print(json.dumps(res, indent=1), flush=True)


if __name__ == "__main__":
    main()
