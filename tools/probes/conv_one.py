"""One convolution pass repeated: a standalone target for timing and PMC passes.

    python tools/probes/conv_one.py PASS N H W C Cout k stride pad [reps]
PASS: fwd (with the fused BN statistics) | dgrad (fused BN backward + shortcut gradient when
the geometry keeps the shape) | dgradbn (fused BN backward only) | wgrad.  Prints the per-call device time."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributedtensorflowexample_amd.ops import cnn as CN  # noqa: E402

BF = torch.bfloat16


def main():
    ps = sys.argv[1]
    N, H, W, C, Co, k, s, p = (int(v) for v in sys.argv[2:10])
    reps = int(sys.argv[10]) if len(sys.argv) > 10 else 20
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(N, H, W, C, generator=g).to(BF).to(dev)
    ld = CN.kpad(k, k, C)
    w = (torch.randn(Co, ld, generator=g) * (k * k * C) ** -0.5).to(BF).to(dev)
    OH, OW = CN.out_hw(H, W, k, s, p)
    dy = torch.randn(N, OH, OW, Co, generator=g).to(BF).to(dev)
    cs, cq = torch.zeros(Co, device=dev), torch.zeros(Co, device=dev)
    mean, rstd = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    sdy, sdx = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    dw = torch.zeros(Co, ld, device=dev)
    if ps == "fwd":
        fn = lambda: CN.conv_fwd(x, w, k, k, s, p, colsum=cs, colsq=cq)  # noqa: E731
    elif ps in ("dgrad", "dgradbn"):
        res = x if ps == "dgrad" else None
        fn = lambda: CN.conv_dgrad(dy, w, x.shape, k, k, s, p, residual=res,  # noqa: E731
                                   bn=(x, x, mean, rstd, sdy, sdx))
    else:
        fn = lambda: CN.conv_wgrad(dy, x, dw, k, k, s, p)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    print(json.dumps({"pass": ps, "shape": sys.argv[2:10], "us": round(e0.elapsed_time(e1) * 1e3 / reps, 1)}),
          flush=True)


if __name__ == "__main__":
    main()
