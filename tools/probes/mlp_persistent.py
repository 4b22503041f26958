"""Persistent single-launch MLP engine vs the two-launch pipelined step (hipGraph replay and
C++ host loop): us/step at K = 20 / 200 / 2000 / 20000 steps, median of 3, one JSON line per K.
"""
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
    dev = torch.device("cuda:0")
    p = init_params(dev, seed=1234)
    x, y = mnist_like_device(55000, seed=100, device=dev)
    tr = FusedMLPTrainer(p, x, y, 100, 0.001)
    tr.run(200)
    tr.run_persistent(200)
    tr.run_launched(50)
    tr.flush()
    torch.cuda.synchronize()
    tr.check()
    for k in [int(a) for a in sys.argv[1:]] or (20, 200, 2000, 20000):
        res = {"K": k}
        for mode in ("graph", "host", "persistent"):
            if mode == "host" and k > 2000:
                continue
            ts = []
            for _ in range(3):
                if mode == "graph":
                    tr.flush()
                    tr.run(1, use_graph=False)  # graphs replay from a pending state
                    tr.prepare(k)
                else:
                    tr.flush()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                if mode == "graph":
                    tr.run(k)
                elif mode == "host":
                    tr.run_launched(k)
                else:
                    tr.run_persistent(k)
                tr.flush()
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) * 1e6 / k)
            res[mode + "_us_per_step"] = round(sorted(ts)[1], 3)
        tr.check()
        res["persistent_samples_per_s"] = round(100 / res["persistent_us_per_step"] * 1e6)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
