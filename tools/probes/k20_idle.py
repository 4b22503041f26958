"""Driver-sized timed region (bench.py --steps 20, host-loop launch) vs how long the GPU sat
idle before it: the region exactly as bench.py brackets it (synchronize, clock, 20 steps + the
flush launched by the same call, synchronize, clock), preceded by
  warm_N : N untimed steps issued just before the opening synchronize (no idle gap),
  idle_S : the device idle for S seconds first (time.sleep after a synchronize).
Medians over REPS interleaved repetitions, us per step.

    python tools/probes/k20_idle.py   (env K=20, REPS=9)
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


def main():
    dev = torch.device("cuda:0")
    K = int(os.environ.get("K", "20"))
    reps = int(os.environ.get("REPS", "9"))
    x, y = mnist_like_device(55000, seed=100, device=dev)
    tr = FusedMLPTrainer(init_params(dev, seed=1234), x, y)
    tr.run(5)
    tr.run_launched(200)
    tr.flush()
    tr.run_launched(1)

    def region():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.run_launched(K, flush=True)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e6 / K
        tr.run_launched(1)  # an update pending again, as after the warmup
        return dt

    cases = {
        "warm_40": lambda: tr.run_launched(40),
        "warm_8": lambda: tr.run_launched(8),
        "idle_0.0001": lambda: (torch.cuda.synchronize(), time.sleep(1e-4)),
        "idle_0.001": lambda: (torch.cuda.synchronize(), time.sleep(1e-3)),
        "idle_0.01": lambda: (torch.cuda.synchronize(), time.sleep(1e-2)),
        "idle_0.1": lambda: (torch.cuda.synchronize(), time.sleep(1e-1)),
    }
    res = {k: [] for k in cases}
    for _ in range(reps):
        for name, pre in cases.items():
            pre()
            res[name].append(region())
    out = {k: {"med_us_per_step": round(sorted(v)[len(v) // 2], 3), "min": round(min(v), 3)}
           for k, v in res.items()}
    # the per-launch host cost of the C++ loop: issue 2000 steps without waiting
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.run_launched(2000)
    t_issue = (time.perf_counter() - t0) * 1e6 / 2000
    torch.cuda.synchronize()
    out["host_issue_us_per_step"] = round(t_issue, 3)
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
