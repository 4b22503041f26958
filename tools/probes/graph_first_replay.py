"""Is the first replay of a freshly captured MLP hipGraph slower than later replays of the
same graph?  (The timed region of a short bench run replays a graph captured just before
the clock.)  Times, for K = 20 steps: first replay of a fresh graph, then 3 more replays of
it (same batches again: timing only), over 5 fresh graphs; medians in us per step."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from distributedtensorflowexample_amd.data.synthetic import mnist_like_device  # noqa: E402
from distributedtensorflowexample_amd.models.mlp import init_params  # noqa: E402
from distributedtensorflowexample_amd.train.fused_mlp import FusedMLPTrainer  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda:0")
    p = init_params(dev, seed=1234)
    x, y = mnist_like_device(55000, seed=100, device=dev)
    tr = FusedMLPTrainer(p, x, y, 100, 0.001)
    tr.run(200)
    first, later = [], []
    for _ in range(5):
        tr.prepare(k)
        g = tr._graph(k)
        for i in range(4):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g.replay()
            torch.cuda.synchronize()
            (first if i == 0 else later).append((time.perf_counter() - t0) * 1e6 / k)
        tr.pos = (tr.pos + k) % tr.nbatches
        tr.cur ^= k & 1
        tr.run(1, use_graph=False)
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    print(json.dumps({"K": k, "first_replay_us_per_step": round(med(first), 3),
                      "later_replay_us_per_step": round(med(later), 3),
                      "first_all": [round(v, 2) for v in first]}), flush=True)


if __name__ == "__main__":
    main()
