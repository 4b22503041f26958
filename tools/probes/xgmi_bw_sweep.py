"""Bus-bandwidth sweep of the bandwidth-mode xGMI all-reduce (protocol "bw") and the LL
two-shot (push2) on ONE GPU with simulated local peers.

LOCAL-PEER NUMBERS: every "peer" slot is HBM of the same GPU and every peer flag is
pre-raised, so one rank's kernel runs alone and moves exactly the bytes it would move in a
W-rank job (its sends into the W-1 peer slots, the owner sum, the gathers) -- but over the
local memory system, not over xGMI.  They bound the kernel's own overhead (launch, flags,
instruction issue, the UC-memory traffic pattern); the xGMI numbers come from the 8-GPU node
(parallel/select.py times bw against RCCL per bucket size there).

    python tools/probes/xgmi_bw_sweep.py [--out gpurun_out/xgmi_bw_sweep.jsonl]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributedtensorflowexample_amd.parallel.xgmi import XgmiComm  # noqa: E402

XG_BLOCKS = 256


def raise_all_flags(comm, regs, protocol):
    """Pre-raise every flag / epoch word a rank could wait for (epoch 0x7fffffff)."""
    W, S = comm.world_size, comm.slot_stride
    if protocol == "bw":
        CS = ((S + W - 1) // W + 3) // 4 * 4
        f0 = 2 * W * CS + 2 * S
        for r in regs:
            r.view(torch.int32)[f0:f0 + 2 * W * XG_BLOCKS] = 0x7FFFFFFF
    else:  # LL words: epoch in the high half of every word
        for r in regs:
            r.fill_(0x7FFFFFFF << 32)


def time_calls(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/xgmi_bw_sweep.jsonl")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    rows = []
    for mb in (1, 4, 16, 32, 64, 128):
        n = mb * (1 << 20) // 4
        x = torch.randn(n, device=dev)
        y = torch.empty_like(x)
        t_copy = time_calls(lambda: y.copy_(x))
        for W in (2, 4, 8):
            for proto in ("bw",):
                if proto == "push2" and mb > 32:
                    continue  # LL words: 8 B per element per slot; large buckets are bw's
                comm, regs = XgmiComm.with_local_peers(0, W, n, device=dev, protocol=proto,
                                                       timeout_s=5.0)
                raise_all_flags(comm, regs, proto)
                t = time_calls(lambda: comm.allreduce_sum_(x))
                comm.check()
                algbw = n * 4 / t / 1e3  # GB/s
                r = {"protocol": proto, "world": W, "MB": mb, "us": round(t, 1),
                     "algbw_GBs": round(algbw, 1),
                     "busbw_GBs": round(algbw * 2 * (W - 1) / W, 1),
                     "copy_us": round(t_copy, 1),
                     "note": "local peers on one GPU (not xGMI)"}
                rows.append(r)
                print(json.dumps(r), flush=True)
                comm.destroy()
                del regs
                torch.cuda.empty_cache()
    with open(a.out, "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
