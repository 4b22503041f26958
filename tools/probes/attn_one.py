"""BERT-base attention (batch 128, seq 128, 12 heads x 64) forward + backward, repeated:
a standalone target for timing and PMC passes of attn_fwd_kernel / attn_bwd_kernel.

    python tools/probes/attn_one.py [reps] [batch] [seq]
prints the per-call device time of each kernel from torch.cuda events.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributedtensorflowexample_amd.ops import transformer as TR  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    S = int(sys.argv[3]) if len(sys.argv) > 3 else 128
    nh, D = 12, 64
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    qkv = (torch.randn(B * S, 3 * nh * D, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    dout = (torch.randn(B * S, nh * D, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    o, lse = TR.attn_fwd(qkv, B, S, nh)
    TR.attn_bwd(qkv, o, dout, lse, B, S, nh)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ev[0].record()
    for _ in range(reps):
        o, lse = TR.attn_fwd(qkv, B, S, nh)
    ev[1].record()
    for _ in range(reps):
        TR.attn_bwd(qkv, o, dout, lse, B, S, nh)
    ev[2].record()
    ev[2].synchronize()
    print(json.dumps({"B": B, "S": S, "fwd_us": round(ev[0].elapsed_time(ev[1]) * 1e3 / reps, 2),
                      "bwd_us": round(ev[1].elapsed_time(ev[2]) * 1e3 / reps, 2)}), flush=True)


if __name__ == "__main__":
    main()
