"""LayerNorm backward at the BERT shape (16384 x 768, residual gradient and column sums
fused): row slots per wave 2 (default) vs 3 (DTFX_LN_SLOTS=3) vs the H = 768 kernel
(DTFX_LN_H768=1, 16 waves per CU), interleaved, us per call and
the HBM rate of its 4 x 25.2 MB of row traffic.  One JSON line.

    python tools/probes/ln_bwd_slots.py [--rows 16384 --hidden 768 --iters 200 --rounds 5]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from distributedtensorflowexample_amd.ops import _ext
from distributedtensorflowexample_amd.ops import transformer as T


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=16384)
    ap.add_argument("--hidden", type=int, default=768)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    Tn, H = a.rows, a.hidden
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(Tn, H, device=dev, generator=g).to(torch.bfloat16)
    gamma, beta = torch.ones(H, device=dev), torch.zeros(H, device=dev)
    _, mean, rstd = T.layernorm_fwd(x, gamma, beta)
    dy = torch.randn(Tn, H, device=dev, generator=g).to(torch.bfloat16)
    dres = torch.randn(Tn, H, device=dev, generator=g).to(torch.bfloat16)
    dg, db, ds = (torch.zeros(H, device=dev) for _ in range(3))
    hip = _ext.hip()
    res = {2: [], 3: [], "h768": []}
    try:
        for _ in range(a.rounds):
            for slots in (2, 3, "h768"):
                hip.ln_bwd_set_slots(2 if slots == "h768" else slots)
                hip.ln_bwd_set_h768(1 if slots == "h768" else 0)
                for _ in range(10):
                    T.layernorm_bwd(dy, x, mean, rstd, gamma, dg, db, dres, dxsum=ds)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    T.layernorm_bwd(dy, x, mean, rstd, gamma, dg, db, dres, dxsum=ds)
                e1.record()
                torch.cuda.synchronize()
                res[slots].append(e0.elapsed_time(e1) * 1e3 / a.iters)
    finally:
        hip.ln_bwd_set_slots(-1)
        hip.ln_bwd_set_h768(-1)
    # what the default kernel's time is made of: without the column sums (1/3 of the
    # cross-block atomics) and without the residual gradient (1/4 of the row traffic)
    parts = {}
    for name, kw in (("full", dict(dres=dres, dxsum=ds)), ("no_dxsum", dict(dres=dres)),
                     ("no_dres", dict(dxsum=ds)), ("neither", {})):
        v = []
        for _ in range(a.rounds):
            for _ in range(10):
                T.layernorm_bwd(dy, x, mean, rstd, gamma, dg, db, **kw)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                T.layernorm_bwd(dy, x, mean, rstd, gamma, dg, db, **kw)
            e1.record()
            torch.cuda.synchronize()
            v.append(e0.elapsed_time(e1) * 1e3 / a.iters)
        parts[name] = round(sorted(v)[len(v) // 2], 2)
    nbytes = 4 * Tn * H * 2
    out = {"rows": Tn, "hidden": H, "iters": a.iters, "default_slots_us": parts}
    for s, v in res.items():
        med = sorted(v)[len(v) // 2]
        out["slots%s" % s] = {"us_median": round(med, 2), "all": [round(t, 2) for t in v],
                              "TB_per_s": round(nbytes / med / 1e6, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
