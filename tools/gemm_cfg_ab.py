"""A/B of the bf16 GEMM tile configurations on the BERT-base training shapes and squares, in
ONE process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24), random operands.

    python tools/gemm_cfg_ab.py [--cfgs 0,3,5] [--rounds 5]

Prints one JSON line per shape: TFLOP/s (median over rounds) per configuration plus
hipBLASLt (torch.matmul) and the max error of config 5 against an f32 reference.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedtensorflowexample_amd.ops import bf16, hip  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="0,5,6")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--shapes", default="all")
    a = ap.parse_args()
    cfgs = [int(c) for c in a.cfgs.split(",")]
    dev = torch.device("cuda:0")
    T = 128 * 128
    shapes = [  # (name, M, N, K, ta, tb, epilogue)
        ("qkv_fwd", T, 2304, 768, False, True, None), ("out_fwd", T, 768, 768, False, True, None),
        ("ffn1_fwd_gelu", T, 3072, 768, False, True, "gelu"),
        # epilogue cost split of the GELU shapes (same GEMM, epilogue variants)
        ("ffn1_fwd_plain", T, 3072, 768, False, True, None),
        ("ffn1_fwd_bias", T, 3072, 768, False, True, "bias"),
        ("ffn1_fwd_gelu_noaux", T, 3072, 768, False, True, "gelu_noaux"),
        ("ffn2_dgrad_plain", T, 3072, 768, False, False, None),
        ("ffn2_fwd", T, 768, 3072, False, True, None),
        ("qkv_dgrad", T, 768, 2304, False, False, None), ("ffn1_dgrad", T, 768, 3072, False, False, None),
        ("ffn2_dgrad_gelu", T, 3072, 768, False, False, "gelu_grad"),
        ("ffn1_wgrad", 3072, 768, T, True, False, "f32"), ("qkv_wgrad", 2304, 768, T, True, False, "f32"),
        # the MLM decoder at batch 128 (2432 masked rows, vocabulary padded to 30528):
        # logits, hidden-state gradient, weight gradient
        ("dec_fwd", 2432, 30528, 768, False, True, None), ("dec_dgrad", 2432, 768, 30528, False, False, None),
        ("dec_wgrad", 30528, 768, 2432, True, False, "f32"),
        ("sq4096", 4096, 4096, 4096, False, True, None), ("sq8192", 8192, 8192, 8192, False, True, None),
        # ResNet-50 1x1 convolutions at batch 256 as plain GEMMs (x [pixels][Cin] W[Cout][Cin]^T)
        ("r_l3c3_fwd", 50176, 1024, 256, False, True, None), ("r_l2c3_fwd", 200704, 512, 128, False, True, None),
        ("r_l3c1_fwd", 50176, 256, 1024, False, True, None), ("r_l4c3_fwd", 12544, 2048, 512, False, True, None),
        ("r_l1c3_fwd", 802816, 256, 64, False, True, None), ("r_l4c1_fwd", 12544, 512, 2048, False, True, None)]
    if a.shapes != "all":
        keep = a.shapes.split(",")
        shapes = [s for s in shapes if s[0] in keep]
    h = hip()
    for name, M, N, K, ta, tb, epi in shapes:
        x = (torch.rand(*((K, M) if ta else (M, K)), device=dev) * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(*((N, K) if tb else (K, N)), device=dev) * 2 - 1).to(torch.bfloat16)
        kw = {}
        if epi == "f32":
            out = torch.zeros(M, N, device=dev)
            kw = dict(out=out, beta=1.0)
        elif epi == "gelu":
            kw = dict(bias=torch.zeros(N, device=dev), act="gelu",
                      aux_out=torch.empty(M, N, device=dev, dtype=torch.bfloat16),
                      out=torch.empty(M, N, device=dev, dtype=torch.bfloat16))
        elif epi == "bias":
            kw = dict(bias=torch.zeros(N, device=dev),
                      out=torch.empty(M, N, device=dev, dtype=torch.bfloat16))
        elif epi == "gelu_noaux":
            kw = dict(bias=torch.zeros(N, device=dev), act="gelu",
                      out=torch.empty(M, N, device=dev, dtype=torch.bfloat16))
        elif epi == "gelu_grad":
            kw = dict(act_grad="gelu", aux_in=torch.zeros(M, N, device=dev, dtype=torch.bfloat16),
                      out=torch.empty(M, N, device=dev, dtype=torch.bfloat16))
        else:
            kw = dict(out=torch.empty(M, N, device=dev, dtype=torch.bfloat16))
        A = x.t() if ta else x
        B = w.t() if tb else w
        lib_out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        res = {c: [] for c in cfgs}
        res["hipblaslt"] = []
        for _ in range(a.rounds):
            for c in cfgs:
                h.gemm_bf16_set_cfg(c)
                res[c].append(timeit(lambda: bf16.gemm(x, w, ta, tb, **kw)))
            res["hipblaslt"].append(timeit(lambda: torch.matmul(A, B, out=lib_out)))
        h.gemm_bf16_set_cfg(-1)
        res["auto"] = [timeit(lambda: bf16.gemm(x, w, ta, tb, **kw)) for _ in range(a.rounds)]
        fl = 2.0 * M * N * K
        line = {"shape": name, "M": M, "N": N, "K": K}
        for k, v in res.items():
            line["tflops_%s" % k] = round(fl / sorted(v)[len(v) // 2] / 1e12, 1)
        for c in (5, 6):
            if c in cfgs and epi is None:
                h.gemm_bf16_set_cfg(c)
                y = bf16.gemm(x, w, ta, tb, out_dtype=torch.float32)
                h.gemm_bf16_set_cfg(-1)
                line["err%d" % c] = float((y - A.float() @ B.float()).abs().max())
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
