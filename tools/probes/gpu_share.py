"""How several async-PS workers sharing ONE GPU contend on it: N workers each loop the fused
worker's GPU step shape -- the three reference-MLP step kernels + a stream synchronize (what
``mlp_ps_worker_step`` does per step, minus the PS RPC) -- as N PROCESSES (the reference's
layout: one OS process per worker, run_single_gpu.sh / run_multi_gpu.sh) or as N THREADS of one
process (one HIP context, a stream per worker).  Aggregate steps/s per layout and N.

    python tools/probes/gpu_share.py --n 1,2,4,8 --secs 3
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def _setup():
    import torch

    from distributedtensorflowexample_amd.data.synthetic import mnist_like_device
    from distributedtensorflowexample_amd.models.mlp import init_params
    from distributedtensorflowexample_amd.ops import mlp_step

    dev = torch.device("cuda:0")
    p = init_params(dev, seed=0)
    x, y = mnist_like_device(100, seed=1, device=dev)
    ws = mlp_step.StepWorkspace(100, dev)
    g = torch.zeros_like(p)
    return torch, mlp_step, p, x, y, ws, g


def _loop(secs, start, stream=None):
    torch, mlp_step, p, x, y, ws, g = _setup()
    s = stream or torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(20):
            mlp_step.step_grad(p, x, y, ws, g)
        s.synchronize()
        if start is not None:
            start.wait()
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < secs:
            mlp_step.step_grad(p, x, y, ws, g)
            s.synchronize()
            n += 1
    return n / (time.perf_counter() - t0)


def _proc(secs, q, start):
    q.put(_loop(secs, start))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="1,2,4,8")
    ap.add_argument("--secs", type=float, default=3.0)
    a = ap.parse_args()
    out = []
    ctx = mp.get_context("spawn")
    for n in [int(v) for v in a.n.split(",")]:
        q, start = ctx.Queue(), ctx.Event()
        ps = [ctx.Process(target=_proc, args=(a.secs, q, start)) for _ in range(n)]
        for p in ps:
            p.start()
        time.sleep(25.0)  # torch import + context creation in every process
        start.set()
        rates = [q.get(timeout=a.secs + 120) for _ in ps]
        for p in ps:
            p.join()
        row = {"layout": "processes", "n": n, "steps_per_s": round(sum(rates), 1)}
        out.append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
    import torch  # noqa: F401  (this process: the threaded layout)

    for n in [int(v) for v in a.n.split(",")]:
        rates, ev = [None] * n, threading.Event()

        def run(i):
            rates[i] = _loop(a.secs, ev)

        ts = [threading.Thread(target=run, args=(i,)) for i in range(n)]
        for t in ts:
            t.start()
        time.sleep(3.0)
        ev.set()
        for t in ts:
            t.join()
        row = {"layout": "threads", "n": n, "steps_per_s": round(sum(rates), 1)}
        out.append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
    print(json.dumps({"note": "fused MLP worker step (3 kernels + stream sync) per worker, one "
                              "MI355X", "rows": out}), flush=True)


if __name__ == "__main__":
    main()
