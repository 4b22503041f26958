"""Achievable HBM bandwidth on this GPU for the access mixes the memory-bound kernels see:
write-only (fill), read-only (sum), read+write (copy) and 1 read : 4 writes, over 512 MB
buffers.  Prints GB/s per mix (the practical ceiling for the roofline's byte bound).

    python tools/probes/hbm_bw.py [MB] [reps]
"""
import json
import sys

import torch


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


def main():
    mb = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    n = mb * (1 << 20) // 2
    dev = torch.device("cuda:0")
    x = torch.randn(n, device=dev).to(torch.bfloat16)
    y = torch.empty_like(x)
    small = torch.empty(n // 4, device=dev, dtype=torch.bfloat16).normal_()
    big = torch.empty(n // 4, 4, device=dev, dtype=torch.bfloat16)
    res = {}
    t = timed(lambda: y.fill_(1.0), reps)
    res["write_GBs"] = round(2 * n / t / 1e9)
    t = timed(lambda: x.sum(), reps)
    res["read_GBs"] = round(2 * n / t / 1e9)
    t = timed(lambda: y.copy_(x), reps)
    res["copy_GBs"] = round(4 * n / t / 1e9)
    t = timed(lambda: big.copy_(small[:, None].expand(-1, 4)), reps)
    res["read1_write4_GBs"] = round((2 * n // 4 + 2 * n) / t / 1e9)
    res["MB"] = mb
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
