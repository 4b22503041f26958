"""The BERT MLM head's logits GEMM (masked tokens x vocab, K = 768, bias, f32 output) under each
bf16 GEMM tile configuration vs the automatic choice (one MI355X).

    python tools/probes/bert_head_gemm.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributedtensorflowexample_amd.models.bert import BertConfig  # noqa: E402
from distributedtensorflowexample_amd.ops import bf16 as B16, hip  # noqa: E402


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
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    V = BertConfig().vocab_padded  # the model's padded vocabulary (row stride % 8 == 0)
    for M in (2432, 2458, 4915):
        x = torch.randn(M, 768, device=dev).to(torch.bfloat16)
        E = torch.randn(V, 768, device=dev).mul_(0.02).to(torch.bfloat16)
        b = torch.zeros(V, device=dev)
        res = {"M": M, "N": V, "K": 768}
        for cfg in (-1, 0, 5, 6):
            hip().gemm_bf16_set_cfg(cfg)
            us = timeit(lambda: B16.gemm(x, E, False, True, bias=b, out_dtype=torch.float32))
            res["us_cfg%d" % cfg if cfg >= 0 else "us_auto"] = round(us, 1)
        hip().gemm_bf16_set_cfg(-1)
        res["tflops_auto"] = round(2 * M * V * 768 / res["us_auto"] * 1e-6, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
