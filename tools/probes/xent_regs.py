"""MLM cross-entropy at the BERT shape (2432 masked rows x 30522 classes, bf16 logits and
dlogits, ld 30528): the row held in registers (DTFX_XENT_REGS=1, one read of the logits) vs the
two-pass kernel, interleaved; us per call and the rate of its minimum traffic (one read + one
write of the [rows x ld] bf16 product).  One JSON line.

    python tools/probes/xent_regs.py [--rows 2432 --iters 100 --rounds 5]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from distributedtensorflowexample_amd.ops import _ext  # noqa: E402
from distributedtensorflowexample_amd.ops import transformer as T  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2432)
    ap.add_argument("--classes", type=int, default=30522)
    ap.add_argument("--ld", type=int, default=30528)
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    logits = (torch.randn(a.rows, a.ld, device=dev, generator=g) * 3).to(torch.bfloat16)
    lab = torch.randint(0, a.classes, (a.rows,), device=dev, dtype=torch.int32)
    hip = _ext.hip()
    res = {0: [], 1: []}
    outs = {}
    try:
        for _ in range(a.rounds):
            for regs in (0, 1):
                hip.xent_set_regs(regs)
                for _ in range(5):
                    outs[regs] = T.mlm_xent(logits, lab, a.classes, 1.0 / a.rows)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    T.mlm_xent(logits, lab, a.classes, 1.0 / a.rows)
                e1.record()
                torch.cuda.synchronize()
                res[regs].append(e0.elapsed_time(e1) * 1e3 / a.iters)
    finally:
        hip.xent_set_regs(-1)
    nbytes = 2 * a.rows * a.ld * 2
    out = {"rows": a.rows, "classes": a.classes, "ld": a.ld, "iters": a.iters,
           "max_abs_diff": {"loss": float((outs[0][0] - outs[1][0]).abs().max()),
                            "dlogits": float((outs[0][2].float() - outs[1][2].float()).abs().max()),
                            "correct_equal": bool(torch.equal(outs[0][1], outs[1][1]))}}
    for r, v in res.items():
        med = sorted(v)[len(v) // 2]
        out["regs%d" % r] = {"us_median": round(med, 2), "all": [round(t, 2) for t in v],
                             "TB_per_s": round(nbytes / med / 1e6, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
