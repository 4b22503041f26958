"""Fixed costs of the driver-sized timed region on the C++ host-loop path (bench.py --steps 20
--launch host): wall time vs the GPU-side span (events) of run_launched(K) + flush().

    python tools/probes/k20_host.py   (env K=20, REPS=7)
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
    reps = int(os.environ.get("REPS", "7"))
    x, y = mnist_like_device(55000, seed=100, device=dev)
    tr = FusedMLPTrainer(init_params(dev, seed=1234), x, y)
    tr.run(5)
    tr.run_launched(50)
    tr.flush()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def span(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6, e0.elapsed_time(e1) * 1e3

    res = {}
    for name, fn in [
        ("empty", lambda: None),
        ("run%d+flush" % K, lambda: (tr.run_launched(K), tr.flush())),
        ("run%d_flush_in_call" % K, lambda: tr.run_launched(K, flush=True)),
        ("run%d" % K, lambda: tr.run_launched(K)),
        ("flush", lambda: tr.flush()),
        ("run1+flush", lambda: (tr.run_launched(1), tr.flush())),
        ("run2+flush", lambda: (tr.run_launched(2), tr.flush())),
        ("run%d+flush" % (2 * K), lambda: (tr.run_launched(2 * K), tr.flush())),
    ]:
        w, g = [], []
        for _ in range(reps):
            a, b = span(fn)
            w.append(a)
            g.append(b)
            tr.run_launched(1)  # leave an update pending, as in the bench
        w.sort()
        g.sort()
        res[name] = {"wall_med": round(w[len(w) // 2], 2), "wall_min": round(w[0], 2),
                     "gpu_med": round(g[len(g) // 2], 2)}
    # bare sync round trip (no events)
    ws = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        ws.append((time.perf_counter() - t0) * 1e6)
    res["sync_only_us"] = round(sorted(ws)[len(ws) // 2], 2)
    print(json.dumps(res, indent=1), flush=True)


if __name__ == "__main__":
    main()
