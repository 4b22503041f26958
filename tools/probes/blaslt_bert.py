"""Per-call A/B of the BERT-base layer GEMMs: this repo's bf16 kernel (with the epilogue the model
uses) vs the hipBLASLt call that computes the same output in one library GEMM (torch.addmm with
the residual or the bias as C, torch.mm when there is no epilogue).  One process, interleaved
rounds, random operands; prints one JSON line per call with the median us of both and the max
abs difference.

    python tools/probes/blaslt_bert.py [--tokens 16384] [--rounds 7]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributedtensorflowexample_amd.ops import bf16 as B16  # noqa: E402


def timeit(fn, iters=20):
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
    ap.add_argument("--tokens", type=int, default=128 * 128)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--head", action="store_true", help="the decoder GEMMs instead of the layer's")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    T, H, F = a.tokens, 768, 3072
    g = torch.Generator(device=dev).manual_seed(0)

    def r(*shape):
        return (torch.randn(*shape, device=dev, generator=g) * 0.5).to(torch.bfloat16)

    x, ctx, h1, gact = r(T, H), r(T, H), r(T, H), r(T, F)
    df, da, du, dqkv = r(T, H), r(T, H), r(T, F), r(T, 3 * H)
    Wqkv, Wo, Wi, Wo2 = r(3 * H, H), r(H, H), r(F, H), r(H, F)
    bqkv, bo, bo2 = r(3 * H).float(), r(H).float(), r(H).float()  # the model keeps biases f32
    bqkv16, bo16, bo216 = bqkv.bfloat16(), bo.bfloat16(), bo2.bfloat16()  # addmm wants C's dtype
    calls = {  # name: (ours, hipBLASLt)
        "qkv_fwd_bias": (lambda: B16.gemm(x, Wqkv, False, True, bias=bqkv),
                         lambda: torch.addmm(bqkv16, x, Wqkv.t())),
        "out_fwd_bias_res": (lambda: B16.gemm(ctx, Wo, False, True, bias=bo, residual=x),
                             lambda: torch.addmm(x, ctx, Wo.t()).add_(bo16)),
        "ffn2_fwd_bias_res": (lambda: B16.gemm(gact, Wo2, False, True, bias=bo2, residual=h1),
                              lambda: torch.addmm(h1, gact, Wo2.t()).add_(bo216)),
        "ffn1_dgrad_res": (lambda: B16.gemm(du, Wi, residual=df), lambda: torch.addmm(df, du, Wi)),
        "out_dgrad": (lambda: B16.gemm(da, Wo), lambda: torch.mm(da, Wo)),
        "qkv_dgrad_res": (lambda: B16.gemm(dqkv, Wqkv, residual=da), lambda: torch.addmm(da, dqkv, Wqkv)),
    }
    if a.head:  # the MLM decoder: masked rows x padded vocabulary
        Tm, V = int(T * 0.15) // 64 * 64, 30528
        tn, dlog, E = r(Tm, H), r(Tm, V), r(V, H)
        bdec = r(V).float()
        bdec16 = bdec.bfloat16()
        from distributedtensorflowexample_amd.ops import transformer as TR
        calls = {
            "logits_bias_bf16": (lambda: B16.gemm(tn, E, False, True, bias=bdec),
                                 lambda: torch.addmm(bdec16, tn, E.t())),
            "decoder_dgrad_bf16": (lambda: TR.cast_bf16(B16.gemm(dlog, E, out_dtype=torch.float32)),
                                   lambda: torch.mm(dlog, E)),
            "transform_dgrad": (lambda: B16.gemm(tn, Wo), lambda: torch.mm(tn, Wo)),
        }
    for name, (ours, lt) in calls.items():
        err = (ours().float() - lt().float()).abs().max().item()
        to, tl = [], []
        for _ in range(a.rounds):
            to.append(timeit(ours))
            tl.append(timeit(lt))
        to.sort()
        tl.sort()
        print(json.dumps({"call": name, "tokens": T, "ours_us": round(to[len(to) // 2], 2),
                          "hipblaslt_us": round(tl[len(tl) // 2], 2),
                          "ours_range": [round(to[0], 2), round(to[-1], 2)],
                          "hipblaslt_range": [round(tl[0], 2), round(tl[-1], 2)],
                          "max_abs_diff": err}), flush=True)


if __name__ == "__main__":
    main()
