"""Local cost of the MLP data-parallel engines at world 2 / 4 / 8 on ONE GPU.

Each engine's kernels of rank W-1 run with simulated local peers (``XgmiComm.with_local_peers``)
whose words are pre-staged for epoch 1, and the communicator's epoch counters are reset to 0
before every step, so every in-kernel wait is satisfied at its first poll: what is timed is
the step's local work at that world size -- the larger K of the factor engines' W1 update
(every rank's factors x every rank's batch), the LL words pushed to W-1 peer slots (here local
HBM, not xGMI), the gathers -- without any cross-GPU latency.  Compared against the 1-GPU
two-launch step.  Per-step us of a 400-step hipGraph, the epoch-reset memsets subtracted.

    python tools/probes/engine_local_cost.py > profiles/r3/engine_local_cost.json
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributedtensorflowexample_amd.data.synthetic import mnist_like_device  # noqa: E402
from distributedtensorflowexample_amd.models.mlp import init_params  # noqa: E402
from distributedtensorflowexample_amd.ops import mlp_step  # noqa: E402
from distributedtensorflowexample_amd.ops._ext import hip, ptr, stream_handle  # noqa: E402
from distributedtensorflowexample_amd.parallel.xgmi import XgmiComm  # noqa: E402

STEPS = 400


def graph_us(fn, dev):
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(STEPS):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / STEPS)
    return best


def main():
    dev = torch.device("cuda:0")
    h = hip()
    B = 100
    p = [init_params(dev, 0, stddev=0.3), torch.empty(mlp_step.NPARAM, device=dev)]
    p[1].copy_(p[0])
    out = {}
    # 1-GPU reference: the bench's two-launch step
    x, y = mnist_like_device(2 * B, seed=1, device=dev)
    xp, xc, yc = x[:B], x[B:], y[B:]
    ws = mlp_step.StepWorkspace(B, dev)

    def single():
        h.mlp_fwdapply(ptr(p[0]), ptr(p[1]), 1e-4, ptr(xp), ptr(xc), ptr(ws.buf), ptr(ws.ctr),
                       ptr(ws.stats), ws.stats_ring, B, 1, stream_handle())
        h.mlp_head2(ptr(p[1]), ptr(yc), ptr(ws.buf), B, stream_handle())

    out["single_gpu_2launch_us"] = round(graph_us(single, dev), 2)
    engines = [e for e in os.environ.get("ENGINES", "fused2,fused2x,factor2,fused,factor").split(",") if e]
    for W in (2, 4, 8):
        r = W - 1
        x_all = torch.stack([mnist_like_device(2 * B, seed=10 + q, device=dev)[0]
                             for q in range(W)]).contiguous()
        dz1A = torch.zeros(W * mlp_step.factor_plane(B), device=dev)
        xs = x_all.stride(0)
        res = {}
        for name in engines:
            # each engine's communicator has the slot size the selector gives it
            # (mlp_step.engine_slot_words); "<engine>@big" forces the fused2 pair layout's size
            kind, _, big = name.partition("@")
            words = mlp_step.XG_SLOT_WORDS if big else mlp_step.engine_slot_words(kind)
            comm, regs = XgmiComm.with_local_peers(r, W, words, device=dev, protocol="push",
                                                   timeout_s=1.0)
            S = comm.slot_stride
            word = (1 << 32) | int(torch.tensor([1e-3]).view(torch.int32).item())
            for q in range(W):
                if q != r:
                    o = (1 * W + q) * S  # parity 1 = epoch 1
                    regs[r][o:o + S] = word
            regs[r][(2 * W + 1) * S:(2 * W + 2) * S] = word  # two-shot results (parity 1)
            hx = comm._h

            def reset():
                hx.reset_epochs(stream_handle())

            def fused2():
                reset()
                comm.mlp_fwdapply(p[0], p[1], 1e-4, x_all[r][:B], x_all[r][B:], ws, True)
                h.mlp_head2(ptr(p[1]), ptr(yc), ptr(ws.buf), B, stream_handle(), mlp_step.XG_SLABS)

            def fused2x():
                comm.two_shot = True
                reset()
                comm.mlp_fwdapply(p[0], p[1], 1e-4, x_all[r][:B], x_all[r][B:], ws, True)
                h.mlp_head2(ptr(p[1]), ptr(yc), ptr(ws.buf), B, stream_handle(), mlp_step.XG_SLABS)
                comm.two_shot = False

            def factor2():
                reset()
                comm.mlp_fwdapply_factor(p[0], p[1], 1e-4, x_all[r][:B], x_all[r][B:], xs, dz1A,
                                         ws, True)
                comm.mlp_head(p[1], yc, ws, dz1A, nslab=mlp_step.FACTOR_SLABS)

            def fused():
                reset()
                h.mlp_fwd(ptr(p[0]), 0, 0.0, 0, ptr(xc), ptr(ws.buf), B, stream_handle())
                h.mlp_head(ptr(p[0]), 0, 0.0, 0, ptr(yc), ptr(ws.buf), B, stream_handle())
                comm.mlp_wgrad(p[0], 1e-4, xc, ws)

            def factor():
                reset()
                h.mlp_fwd(ptr(p[0]), 0, 0.0, 0, ptr(x_all[r][B:]), ptr(ws.buf), B, stream_handle())
                comm.mlp_head(p[0], yc, ws, dz1A, nslab=7)
                comm.mlp_wgrad_factor(p[0], 1e-4, x_all[r][B:], xs, dz1A, ws)

            def factor2_fwd():  # the factor engine's first launch + the plain head
                reset()
                comm.mlp_fwdapply_factor(p[0], p[1], 1e-4, x_all[r][:B], x_all[r][B:], xs, dz1A,
                                         ws, True)
                h.mlp_head2(ptr(p[1]), ptr(yc), ptr(ws.buf), B, stream_handle(),
                            mlp_step.FACTOR_SLABS)

            def factor2_head():  # the 1-GPU first launch + the factor engine's head
                reset()
                h.mlp_fwdapply(ptr(p[0]), ptr(p[1]), 1e-4, ptr(x_all[r][:B]), ptr(x_all[r][B:]),
                               ptr(ws.buf), ptr(ws.ctr), ptr(ws.stats), ws.stats_ring, B, 1,
                               stream_handle())
                comm.mlp_head(p[1], yc, ws, dz1A, nslab=mlp_step.FACTOR_SLABS)

            fn = {"fused2": fused2, "fused2x": fused2x, "factor2": factor2, "fused": fused,
                  "factor": factor, "factor2_fwd": factor2_fwd, "factor2_head": factor2_head}[kind]
            t_reset = graph_us(reset, dev)
            res[name] = round(graph_us(fn, dev) - t_reset, 2)
            comm.check()
            res.setdefault("epoch_reset_us", round(t_reset, 2))
            comm.destroy()
            del regs
        out["world%d" % W] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
