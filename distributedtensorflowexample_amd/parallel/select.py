"""Choice of the all-reduce backend for the latency-bound MLP gradient.

``pick_small_allreduce`` creates the xGMI one-shot communicator, verifies it
against RCCL on a random gradient (every rank must agree), times both inside a
captured hipGraph (max over ranks) and returns the faster -- falling back to
RCCL whenever xGMI is unavailable, wrong or slower.  Used by ``bench.py`` and
the mirrored MLP trainer for N > 1.
"""
from __future__ import annotations

import sys
import time

import torch
import torch.distributed as dist

from ..ops import mlp_step
from .xgmi import XgmiComm


def pick_small_allreduce(rccl, mode, world, rank, dev, iters=200, n=None, xgmi_key="dtfx/xgmi/0"):
    """MLP gradient all-reduce backend: the xGMI one-shot kernel when it is available,
    agrees with RCCL on a random gradient, and is faster (mode "auto"); else RCCL.
    Every rank takes the same decision (gloo control plane)."""
    n = mlp_step.NPARAM if n is None else n

    def agree(ok):
        t = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    xg, err = None, ""
    try:
        xg = XgmiComm(rank, world, n, device=dev, key=xgmi_key)
    except Exception as e:  # no IPC / peer mapping on this node
        err = repr(e)
    if not agree(xg is not None):
        print("[bench] xgmi unavailable (%s): RCCL" % err, file=sys.stderr)
        return rccl, None
    g = torch.Generator(device="cpu").manual_seed(1000 + rank)
    ok = True
    try:
        for it in range(10):  # fresh random gradients: both backends must agree every time
            base = torch.randn(n, generator=g).to(dev) * (1 + it)
            ra, xa = base.clone(), base.clone()
            rccl.allreduce_sum_(ra)
            torch.cuda.synchronize()
            dist.barrier()
            xg.allreduce_sum_(xa)
            xg.check()
            ok &= bool(((ra - xa).abs().max() <= 1e-5 * ra.abs().max()).item())
    except Exception as e:
        ok, err = False, repr(e)
    if not agree(ok):
        print("[bench] xgmi failed verification (%s): RCCL" % err, file=sys.stderr)
        return rccl, None
    if mode == "xgmi":
        return xg, None

    def graph_of(c, buf):
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            c.allreduce_sum_(buf)
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(iters):
                c.allreduce_sum_(buf)
        gr.replay()  # warm replay (first-launch costs stay out of the timing)
        torch.cuda.synchronize()
        return gr

    def timed(gr):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gr.replay()
        torch.cuda.synchronize()
        dt = torch.tensor([(time.perf_counter() - t0) / iters * 1e6], dtype=torch.float64)
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        return float(dt.item())

    bufs = [torch.zeros(n, device=dev), torch.zeros(n, device=dev)]
    gr_r, gr_x = graph_of(rccl, bufs[0]), graph_of(xg, bufs[1])
    t_r = t_x = float("inf")
    for _ in range(3):  # interleaved, best of three each
        t_r = min(t_r, timed(gr_r))
        t_x = min(t_x, timed(gr_x))
    xg.check()
    probe = {"rccl": round(t_r, 2), "xgmi": round(t_x, 2)}
    use_x = agree(t_x < t_r)
    if rank == 0:
        print("[bench] small all-reduce probe (us/call, max over ranks): %s -> %s"
              % (probe, "xgmi" if use_x else "rccl"), file=sys.stderr)
    return (xg if use_x else rccl), probe
