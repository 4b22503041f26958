"""Timeline of the two-launch pipelined MLP step (the 1-GPU bench engine) from in-kernel
s_memrealtime stamps (100 MHz; every stamp waits for the wave's outstanding memory ops, so it
marks "everything issued before has landed").

Steps 100 and 101 of a 200-step hipGraph chain run the traced kernels (same code, stamps
added): mlp_fwdapply_kernel<7, 0, true, .., KS> (7 x KS W1-tile blocks x 4 waves: 0 entry,
1 phase-A operands landed, 2 W1 tile applied + barrier, 3 slab stored; 7 small-parameter
blocks: 0, 3; KS = 28, or 14 with DTFX_MLP_KS=14) and mlp_head_kernel<.., KS> (100 one-wave
blocks: 0 entry, 1 operands landed, 2 compute
done, 3 stores landed).  Prints per-phase medians / maxima and the kernel-to-kernel gaps
(the dependent-launch boundaries a single-launch design would have to beat).

    python tools/probes/mlp_pipelined_trace.py > profiles/r3/mlp_trace/pipelined_trace.json
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributedtensorflowexample_amd.models.mlp import init_params  # noqa: E402
from distributedtensorflowexample_amd.ops import hip, mlp_step  # noqa: E402
from distributedtensorflowexample_amd.ops._ext import ptr, stream_handle  # noqa: E402

NB_SMALL = 7


def phases(t, cols):
    """t: [waves, 4] int64 stamps (10 ns) -> per-interval median / max in us."""
    t = t.double()
    t = t[t[:, 0] > 0]
    out = {}
    for a, b, name in cols:
        d = (t[:, b] - t[:, a]) / 100.0
        out[name] = [round(float(d.median()), 3), round(float(d.max()), 3)]
    return out, float(t[:, 0].min()), float(t[:, 0].max()), float(t[:, 3].max())


def main():
    dev = torch.device("cuda:0")
    h = hip()
    NB_W1 = 7 * h.mlp_single_ks()
    B, nb = 100, 550
    p = [init_params(dev, 0), torch.empty(mlp_step.NPARAM, device=dev)]
    x = torch.rand(nb * B, 784, device=dev)
    y = torch.randint(0, 10, (nb * B,), device=dev, dtype=torch.int32)
    ws = mlp_step.StepWorkspace(B, dev)
    trf = [torch.zeros((NB_W1 + NB_SMALL) * 4 * 4, dtype=torch.int64, device=dev) for _ in range(2)]
    trh = [torch.zeros(B * 4, dtype=torch.int64, device=dev) for _ in range(2)]
    lr = 1e-4

    def step(i, cur, traced):
        xb, yb = x[(i % nb) * B:(i % nb + 1) * B], y[(i % nb) * B:(i % nb + 1) * B]
        xp = x[((i - 1) % nb) * B:((i - 1) % nb + 1) * B]
        s = stream_handle()
        if traced is None:
            h.mlp_fwdapply(ptr(p[cur]), ptr(p[cur ^ 1]), lr, ptr(xp), ptr(xb), ptr(ws.buf),
                           ptr(ws.ctr), ptr(ws.stats), ws.stats_ring, B, 1, s)
            h.mlp_head2(ptr(p[cur ^ 1]), ptr(yb), ptr(ws.buf), B, s)
        else:
            h.mlp_pipelined_trace(ptr(p[cur]), ptr(p[cur ^ 1]), lr, ptr(xp), ptr(xb), ptr(yb),
                                  ptr(ws.buf), ptr(ws.ctr), ptr(ws.stats), ws.stats_ring, B, s,
                                  ptr(trf[traced]), ptr(trh[traced]))

    for i in range(20):
        step(i, i & 1, None)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for i in range(200):
            step(i, i & 1, 0 if i == 100 else 1 if i == 101 else None)
    reps = []
    for _ in range(5):
        for t in trf + trh:
            t.zero_()
        g.replay()
        torch.cuda.synchronize()
        fw = [trf[k].view(-1, 4).cpu() for k in range(2)]
        hd = [trh[k].view(-1, 4).cpu() for k in range(2)]
        w1 = [f[:NB_W1 * 4] for f in fw]
        sm = [f[NB_W1 * 4:] for f in fw]
        f_ph, f0, f0max, f_end = phases(w1[0], [(0, 1, "entry->operands_landed"),
                                                (1, 2, "mfma+apply+barrier"),
                                                (2, 3, "phaseB_fwd+slab_store"),
                                                (0, 3, "wave_total")])
        s_ph, _, _, s_end = phases(sm[0], [(0, 3, "small_block_total")])
        h_ph, h0, h0max, h_end = phases(hd[0], [(0, 1, "entry->operands_landed"),
                                                (1, 2, "compute"), (2, 3, "stores_landed"),
                                                (0, 3, "wave_total")])
        _, f1, _, _ = phases(w1[1], [(0, 3, "x")])
        fwd_end = max(f_end, s_end)
        reps.append({
            "fwdapply": dict(f_ph, start_skew_us=round((f0max - f0) / 100, 3),
                             span_us=round((fwd_end - f0) / 100, 3)),
            "fwdapply_small": s_ph,
            "head": dict(h_ph, start_skew_us=round((h0max - h0) / 100, 3),
                         span_us=round((h_end - h0) / 100, 3)),
            "gap_fwd_end_to_head_first_wave_us": round((h0 - fwd_end) / 100, 3),
            "gap_head_end_to_next_fwd_first_wave_us": round((f1 - h_end) / 100, 3),
            "step_period_us(fwd start -> next fwd start)": round((f1 - f0) / 100, 3),
        })
    # untraced reference: the same chain without stamps
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2, stream=s):
        for i in range(200):
            step(i, i & 1, None)
    g2.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g2.replay()
    e1.record()
    torch.cuda.synchronize()
    out = {"k_slices": NB_W1 // 7, "traced_step_replays": reps,
           "untraced_us_per_step": round(e0.elapsed_time(e1) * 1e3 / 1000, 3)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
