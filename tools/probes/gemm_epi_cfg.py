"""BERT-base GEMMs with their real epilogues, timed per tile config.

    DTFX_GEMM_CFG=<0|3|unset> python tools/probes/gemm_epi_cfg.py

One JSON line per case: FFN-in forward (bias + GELU + pre-activation out), FFN-out dgrad
(GELU-grad on the stored pre-activation), QKV forward (bias), FFN-out forward (bias +
residual), plain FFN-in forward without epilogue.
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from distributedtensorflowexample_amd.ops import bf16  # noqa: E402
from tools.gemm_bench import timeit  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    T, Hd, F = 128 * 128, 768, 3072
    bf = torch.bfloat16
    x = torch.randn(T, Hd, device=dev).to(bf)
    w1 = (torch.randn(Hd, F, device=dev) * 0.03).to(bf)
    b1 = torch.randn(F, device=dev) * 0.1
    w2 = (torch.randn(F, Hd, device=dev) * 0.03).to(bf)
    b2 = torch.randn(Hd, device=dev) * 0.1
    wqkv = (torch.randn(Hd, 3 * Hd, device=dev) * 0.03).to(bf)
    bqkv = torch.randn(3 * Hd, device=dev) * 0.1
    u = torch.empty(T, F, device=dev, dtype=bf)
    h = torch.empty(T, F, device=dev, dtype=bf)
    dy = torch.randn(T, Hd, device=dev).to(bf)
    du = torch.empty(T, F, device=dev, dtype=bf)
    y2 = torch.empty(T, Hd, device=dev, dtype=bf)
    qkv = torch.empty(T, 3 * Hd, device=dev, dtype=bf)
    cases = [
        ("ffn_in_fwd_gelu_aux", 2.0 * T * Hd * F,
         lambda: bf16.gemm(x, w1, bias=b1, act="gelu", aux_out=u, out=h)),
        ("ffn_in_fwd_plain", 2.0 * T * Hd * F, lambda: bf16.gemm(x, w1, out=h)),
        ("ffn_out_dgrad_gelugrad", 2.0 * T * Hd * F,
         lambda: bf16.gemm(dy, w2, False, True, act_grad="gelu", aux_in=u, out=du)),
        ("ffn_out_fwd_bias_res", 2.0 * T * Hd * F,
         lambda: bf16.gemm(h, w2, bias=b2, residual=x, out=y2)),
        ("qkv_fwd_bias", 2.0 * T * Hd * 3 * Hd, lambda: bf16.gemm(x, wqkv, bias=bqkv, out=qkv)),
    ]
    cfg = os.environ.get("DTFX_GEMM_CFG", "auto")
    for name, flops, fn in cases:
        t = timeit(fn, iters=30)
        print(json.dumps({"case": name, "cfg": cfg, "us": round(t * 1e6, 1),
                          "tflops": round(flops / t / 1e12, 1)}), flush=True)


if __name__ == "__main__":
    main()
