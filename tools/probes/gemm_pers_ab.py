"""The persistent 8-phase tile loop against one block per tile, interleaved in one process
(``gemm_bf16_set_pers``), per call on the BERT-base shapes it takes (more 256x256 tiles than
CUs) and a square.  Medians of ``--rounds`` interleaved rounds of ``--iters`` calls.

    python tools/probes/gemm_pers_ab.py [--rounds 7]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributedtensorflowexample_amd.ops import bf16  # noqa: E402
from distributedtensorflowexample_amd.ops._ext import hip  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)

    def r(*s):
        return (torch.rand(*s, device=dev, generator=g) - 0.5).to(torch.bfloat16)

    cases = []
    # BERT-base FFN1 forward (X W^T + bias, GELU, pre-activation stored), QKV projection
    # (+ bias), decoder-sized logits, the 16384 x 3072 plain product, 8192^3
    x, w1, b1 = r(16384, 768), r(3072, 768), torch.randn(3072, device=dev)
    aux = torch.empty(16384, 3072, device=dev, dtype=torch.bfloat16)
    cases.append(("ffn1_fwd_gelu_aux 16384x3072x768", 2 * 16384 * 3072 * 768,
                  lambda: bf16.gemm(x, w1, False, True, bias=b1, act="gelu_dsave", aux_out=aux)))
    wq, bq = r(2304, 768), torch.randn(2304, device=dev)
    cases.append(("qkv_fwd_bias 16384x2304x768", 2 * 16384 * 2304 * 768,
                  lambda: bf16.gemm(x, wq, False, True, bias=bq)))
    cases.append(("plain 16384x3072x768", 2 * 16384 * 3072 * 768,
                  lambda: bf16.gemm(x, w1, False, True)))
    xl, wl = r(2560, 768), r(30528, 768)
    cases.append(("logits 2560x30528x768", 2 * 2560 * 30528 * 768,
                  lambda: bf16.gemm(xl, wl, False, True)))
    xs, ws_ = r(8192, 8192), r(8192, 8192)
    cases.append(("plain 8192^3", 2 * 8192 ** 3, lambda: bf16.gemm(xs, ws_, False, True)))
    x4, w4 = r(16384, 768), r(3072, 768)
    out32 = torch.empty(16384, 3072, device=dev)
    cases.append(("f32_out 16384x3072x768", 2 * 16384 * 3072 * 768,
                  lambda: bf16.gemm(x4, w4, False, True, out=out32, out_dtype=torch.float32)))
    old = hip().gemm_bf16_set_pers(1)
    try:
        for name, flop, fn in cases:
            ts = {1: [], 0: []}
            for _ in range(a.rounds):
                for p in (1, 0):
                    hip().gemm_bf16_set_pers(p)
                    ts[p].append(timeit(fn, a.iters))
            med = {p: sorted(v)[len(v) // 2] for p, v in ts.items()}
            print(json.dumps({"case": name, "pers_us": round(med[1], 2), "base_us": round(med[0], 2),
                              "pers_tflops": round(flop / med[1] / 1e6, 1),
                              "base_tflops": round(flop / med[0] / 1e6, 1),
                              "gain_pct": round(100 * (med[0] / med[1] - 1), 2)}), flush=True)
    finally:
        hip().gemm_bf16_set_pers(old)


if __name__ == "__main__":
    main()
