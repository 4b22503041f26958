"""Where the data-parallel MLP engines' extra time goes at world 2 / 4 / 8 (ONE GPU, simulated
peers): in-kernel s_memrealtime stamps of the fused engines' first launch
(mlp_fwdapply_kernel<7, W, TRACE, TWO, 28 slices>), against the same stamps of the 1-GPU
step's first launch.

Set-up as tools/probes/engine_local_cost.py: rank W-1's kernels with local "peer" slots whose
words are pre-staged for epoch 1, the communicator's epochs reset before every step, so every
in-kernel wait is satisfied at its first poll -- the stamps show the kernel's own work per
phase (LL word stores to W-1 peer slots, the gather loads of uncached memory, the second hop
of the two-shot), not xGMI latency.  Per wave (exchanging waves only for 4 / 5 / 6), medians
and maxima in us over the last of several traced steps:

  entry->operands (0->1), MFMA + K-split join (1->4), exchange (4->6; two-shot: hop 1 4->5,
  hop 2 5->6), apply + LDS + barrier (6->2), phase B (2->3), block span (min 0 -> max 3).

    python tools/probes/engine_trace.py > profiles/r4/engine_trace/engine_trace.json
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

B = 100
REPS = 6


def med_max(d):
    d = d[d > -1e8]
    if d.numel() == 0:
        return None
    return [round(float(d.median()), 3), round(float(d.max()), 3)]


def summarize(t, xw, n_small_waves=7 * 4):
    """t: int64 [waves, 8] (xw) or [waves, 4] stamps in 10 ns ticks; the last
    ``n_small_waves`` rows are the small-parameter blocks (dW2 / db1 / db2 + stats)."""
    t = t.double()
    small = t[-n_small_waves:]
    small = small[small[:, 0] > 0]
    w1 = t[:-n_small_waves]
    w1 = w1[w1[:, 0] > 0]
    extra = {}
    if small.numel():
        extra["small_blocks"] = med_max((small[:, 3] - small[:, 0]) / 100.0)
        # per wave role (row % 4): 0 dW2 (half), 1 db1, 2 dW2 half / db2, 3 stats (+ db2)
        sm = t[-n_small_waves:]
        for wv in range(4):
            rows = sm[wv::4]
            rows = rows[rows[:, 0] > 0]
            if rows.numel():
                extra["small_wave%d" % wv] = med_max((rows[:, 3] - rows[:, 0]) / 100.0)
                extra["small_wave%d_start_after_first_us" % wv] = round(
                    float((rows[:, 0].min() - t[t[:, 0] > 0][:, 0].min()) / 100.0), 3)
        extra["small_end_after_w1_end_us"] = round(float((small[:, 3].max() - w1[:, 3].max())
                                                         / 100.0), 3)
    extra["w1_span_us"] = round(float((w1[:, 3].max() - w1[:, 0].min()) / 100.0), 3)
    live = t[:, 0] > 0
    t = t[live]
    us = lambda a, b: (t[:, b] - t[:, a]) / 100.0  # noqa: E731
    out = {"waves": int(t.shape[0])}
    w1 = t[:, 3] > 0
    out["entry_to_operands"] = med_max(us(0, 1)[t[:, 1] > 0])
    out["phaseB"] = med_max(us(2, 3)[w1 & (t[:, 2] > 0)])
    out["span_us"] = round(float((t[:, 3].max() - t[:, 0].min()) / 100.0), 3)
    if xw:
        ex = t[:, 4] > 0
        out["mfma_to_exchange"] = med_max(us(1, 4)[ex])
        out["exchange"] = med_max(us(4, 6)[ex])
        two = ex & (t[:, 5] > 0)
        if bool(two.any()):
            out["hop1"] = med_max(us(4, 5)[two])
            out["hop2"] = med_max(us(5, 6)[two])
        out["apply_barrier"] = med_max(us(6, 2)[ex])
    else:
        out["phaseA_apply_barrier"] = med_max(us(1, 2)[t[:, 2] > 0])
    out.update(extra)
    return out


def main():
    dev = torch.device("cuda:0")
    h = hip()
    p = [init_params(dev, 0, stddev=0.3), torch.empty(mlp_step.NPARAM, device=dev)]
    p[1].copy_(p[0])
    x, y = mnist_like_device(2 * B, seed=1, device=dev)
    xp, xc, yc = x[:B], x[B:], y[B:]
    ws = mlp_step.StepWorkspace(B, dev)
    nblk = mlp_step.HT * 28 + mlp_step.HT if hasattr(mlp_step, "HT") else 7 * 28 + 7
    out = {}
    # 1-GPU step's first launch (the bench engine), 28 slices: [blocks * 4][4]
    ks = int(h.mlp_single_ks())
    trf = torch.zeros((7 * ks + 7) * 4, 4, dtype=torch.int64, device=dev)
    trh = torch.zeros(B * 4, dtype=torch.int64, device=dev)
    for _ in range(REPS):
        trf.zero_()
        h.mlp_pipelined_trace(ptr(p[0]), ptr(p[1]), 1e-4, ptr(xp), ptr(xc), ptr(yc), ptr(ws.buf),
                              ptr(ws.ctr), ptr(ws.stats), ws.stats_ring, B, stream_handle(),
                              ptr(trf), ptr(trh))
        torch.cuda.synchronize()
    out["single"] = summarize(trf.cpu(), False)
    for W in (2, 4, 8):
        r = W - 1
        comm, regs = XgmiComm.with_local_peers(r, W, mlp_step.XG_SLOT_WORDS, device=dev,
                                               protocol="push", timeout_s=1.0)
        S = comm.slot_stride
        word = (1 << 32) | int(torch.tensor([1e-3]).view(torch.int32).item())
        for q in range(W):
            if q != r:
                o = (1 * W + q) * S  # parity 1 = epoch 1
                regs[r][o:o + S] = word
        regs[r][(2 * W + 1) * S:(2 * W + 2) * S] = word  # two-shot results (parity 1)
        tr = torch.zeros((7 * 28 + 7) * 4, 8, dtype=torch.int64, device=dev)
        res = {}
        for name, two in (("fused2", False), ("fused2x", True)):
            comm.two_shot = two
            for _ in range(REPS):
                tr.zero_()
                comm._h.reset_epochs(stream_handle())
                comm.mlp_fwdapply(p[0], p[1], 1e-4, xp, xc, ws, True, trace=tr)
                h.mlp_head2(ptr(p[1]), ptr(yc), ptr(ws.buf), B, stream_handle(),
                            mlp_step.XG_SLABS)
                torch.cuda.synchronize()
            res[name] = summarize(tr.cpu(), True)
        comm.two_shot = False
        comm.check()
        out["world%d" % W] = res
        comm.destroy()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
