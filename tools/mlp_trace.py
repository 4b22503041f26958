"""Timeline of one fused MLP step from in-kernel s_memrealtime stamps (10 ns).

Each wave stamps: 0 entry, 1 operands landed, 2 compute done, 3 stores landed.
One traced step sits in the middle of a graph-replayed chain, so the
measurement sees steady-state boundaries.  Run on the GPU box.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedtensorflowexample_amd.models.mlp import init_params  # noqa: E402
from distributedtensorflowexample_amd.ops import hip, mlp_step  # noqa: E402
from distributedtensorflowexample_amd.ops._ext import ptr, stream_handle  # noqa: E402


def summarize(name, t, nwaves):
    t = t[:nwaves].double()
    ok = t[:, 0] > 0
    t = t[ok]
    t0 = t[:, 0].min()
    r = {"waves": int(ok.sum()),
         "start_skew_p50_p100": [float((t[:, 0] - t0).median() * 10), float((t[:, 0] - t0).max() * 10)],
         "load_p50_p100": [float((t[:, 1] - t[:, 0]).median() * 10), float((t[:, 1] - t[:, 0]).max() * 10)],
         "compute_p50_p100": [float((t[:, 2] - t[:, 1]).median() * 10), float((t[:, 2] - t[:, 1]).max() * 10)],
         "store_p50_p100": [float((t[:, 3] - t[:, 2]).median() * 10), float((t[:, 3] - t[:, 2]).max() * 10)],
         "span_ns": float((t[:, 3].max() - t0) * 10)}
    return name, r, float(t0), float(t[:, 3].max())


def main():
    dev = torch.device("cuda:0")
    h = hip()
    B, nb = 100, 550
    p = init_params(dev, 0)
    x = torch.rand(nb * B, 784, device=dev)
    y = torch.randint(0, 10, (nb * B,), device=dev, dtype=torch.int32)
    ws = mlp_step.StepWorkspace(B, dev)
    tf = torch.zeros(343 * 4, dtype=torch.int64, device=dev)
    th = torch.zeros(100 * 4, dtype=torch.int64, device=dev)
    tw = torch.zeros(98 * 4 * 4, dtype=torch.int64, device=dev)

    def step(i, trace):
        xb, yb = x[(i % nb) * B:(i % nb + 1) * B], y[(i % nb) * B:(i % nb + 1) * B]
        s = stream_handle()
        h.mlp_fwd(ptr(p), 0, 0.0, 0, ptr(xb), ptr(ws.buf), B, s, ptr(tf) if trace else 0)
        h.mlp_head(ptr(p), 0, 0.0, 0, ptr(yb), ptr(ws.buf), B, s, ptr(th) if trace else 0)
        h.mlp_wgrad(ptr(p), 1e-9, 0, ptr(xb), ptr(ws.buf), ptr(ws.ctr), ptr(ws.stats), 4096, B, s,
                    ptr(tw) if trace else 0)

    for i in range(20):
        step(i, False)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for i in range(200):
            step(i, i == 100)
    out = []
    for rep in range(3):
        g.replay()
        torch.cuda.synchronize()
        k1 = summarize("fwd", tf.view(-1, 4).cpu(), 343)
        k2 = summarize("head", th.view(-1, 4).cpu(), 100)
        k3 = summarize("wgrad(typeA)", tw.view(-1, 4).cpu(), 98 * 4)
        res = {k[0]: k[1] for k in (k1, k2, k3)}
        res["gap_fwd_to_head_ns"] = (k2[2] - k1[3]) * 10
        res["gap_head_to_wgrad_ns"] = (k3[2] - k2[3]) * 10
        res["step_span_ns(fwd start..wgrad end)"] = (k3[3] - k1[2]) * 10
        out.append(res)
    # shader clock under (a) an isolated probe, (b) the probe right after the traced chain
    o2 = torch.zeros(2 * 256, dtype=torch.int64, device=dev)
    sink = torch.zeros(1, device=dev)
    clk = {}
    for iters in (1000, 100000):
        h.clock_probe(iters, 256, ptr(o2), ptr(sink), stream_handle())
        torch.cuda.synchronize()
        v = o2.view(-1, 2).double().cpu()
        clk["iters%d_GHz_median" % iters] = float((v[:, 0] / (v[:, 1] * 10)).median())
        clk["iters%d_cycles_per_fma" % iters] = float(v[:, 0].median() / iters)
    g.replay()
    h.clock_probe(1000, 256, ptr(o2), ptr(sink), stream_handle())
    torch.cuda.synchronize()
    v = o2.view(-1, 2).double().cpu()
    clk["after_chain_GHz_median"] = float((v[:, 0] / (v[:, 1] * 10)).median())
    out[-1]["clock"] = clk
    print(json.dumps(out[-1], indent=1))


if __name__ == "__main__":
    main()
