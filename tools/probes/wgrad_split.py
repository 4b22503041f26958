"""Weight-gradient GEMM (A^T, f32 accumulate, split-K): tile config x split factor sweep on
the BERT-base shapes, interleaved rounds in one process."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
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
    dev = torch.device("cuda:0")
    T = 16384
    h = hip()
    for name, M, N in (("ffn", 3072, 768), ("qkv", 2304, 768), ("out", 768, 768)):
        dy = (torch.rand(T, M, device=dev) * 2 - 1).to(torch.bfloat16)
        x = (torch.rand(T, N, device=dev) * 2 - 1).to(torch.bfloat16)
        out = torch.zeros(M, N, device=dev)
        res = {}
        for _ in range(3):
            for cfg, splits in ((0, (0, 2, 3, 4, 6, 8)), (5, (0, 4, 7, 8, 14, 16))):
                h.gemm_bf16_set_cfg(cfg)
                for sk in splits:
                    t = timeit(lambda: bf16.gemm(dy, x, True, False, out=out, beta=1.0, splitk=sk))
                    res.setdefault("cfg%d_split%d" % (cfg, sk), []).append(t)
        h.gemm_bf16_set_cfg(-1)
        fl = 2.0 * M * N * T
        line = {k: round(fl / sorted(v)[1] / 1e12, 1) for k, v in res.items()}
        line["shape"] = name
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
