"""Per-kernel cost of the fused MLP step, measured as hipGraph chains.

For each variant, N dependent launches are captured in one graph and replayed;
time/N is the incremental cost of one launch INCLUDING its kernel boundary,
i.e. exactly what it adds to a training step.  Run on the GPU box:

    python tools/mlp_microbench.py
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedtensorflowexample_amd.models.mlp import init_params  # noqa: E402
from distributedtensorflowexample_amd.ops import hip, mlp_step  # noqa: E402
from distributedtensorflowexample_amd.ops._ext import ptr, stream_handle  # noqa: E402


def chain_time(fn, n=200, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / n)
    return best * 1e6


def main():
    dev = torch.device("cuda:0")
    h = hip()
    B, nb = 100, 550
    p = init_params(dev, 0)
    x = torch.rand(nb * B, 784, device=dev)
    y = torch.randint(0, 10, (nb * B,), device=dev, dtype=torch.int32)
    ws = mlp_step.StepWorkspace(B, dev)
    data = torch.rand(1 << 20, device=dev)
    g = torch.zeros_like(p)
    out = torch.zeros(16, device=dev)
    res = {}
    for mode in (0, 1, 2):
        for grid in (1, 100, 350, 1024):
            res["calib_mode%d_grid%d" % (mode, grid)] = chain_time(
                lambda: h.calib(mode, grid, 64, ptr(ws.ctr), ptr(data), ptr(out), stream_handle()))
    S = lambda: stream_handle()
    xb, yb = x[:B], y[:B]
    res["fwd"] = chain_time(lambda: h.mlp_fwd(ptr(p), 0, 0.0, 0, ptr(xb), ptr(ws.buf), B, S()))
    res["head"] = chain_time(lambda: h.mlp_head(ptr(p), 0, 0.0, 0, ptr(yb), ptr(ws.buf), B, S()))
    res["wgrad_direct"] = chain_time(lambda: h.mlp_wgrad(ptr(p), 1e-9, 0, ptr(xb), ptr(ws.buf),
                                                         ptr(ws.ctr), ptr(ws.stats), 4096, B, S()))
    res["step_direct"] = chain_time(lambda: mlp_step.step_direct(p, xb, yb, ws, 1e-9), n=100)
    res["step_dp_noallreduce"] = chain_time(lambda: mlp_step.step_grad(p, xb, yb, ws, g), n=100)
    print(json.dumps({k: round(v, 3) for k, v in res.items()}, indent=1))


if __name__ == "__main__":
    main()
