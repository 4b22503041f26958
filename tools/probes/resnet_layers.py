"""Per-layer roofline of the ResNet-50 convolutions (batch 256 by default).

Times every convolution of ``models.resnet.conv_specs`` in isolation -- forward with the
fused BN statistics, data gradient (with the fused BN-backward epilogue where the model uses
it, i.e. every conv except the stem and the down-sampling projection) and weight gradient --
and reports time, TFLOP/s, the minimum HBM traffic and the roofline bound
max(FLOP / 2.3 PF/s, bytes / 6.5 TB/s).  One JSON line per (layer, pass), then totals.

    python tools/probes/resnet_layers.py [--batch 256] [--reps 20]   (env ONLY=layer4,layer3.0)
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributedtensorflowexample_amd.models.resnet import conv_specs  # noqa: E402
from distributedtensorflowexample_amd.ops import cnn as CN  # noqa: E402

BF16 = torch.bfloat16
PEAK_FLOPS = 2.3e15
PEAK_BW = 6.5e12


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(3):
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / reps)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    N = a.batch
    size = 56
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0, "bound": 0.0}
    for name, cin, cout, k, s, p in conv_specs():
        H = 224 if name == "conv1" else (size * s if name.endswith("downsample") else size)
        OH, OW = CN.out_hw(H, H, k, s, p)
        if name != "conv1" and name.endswith("conv2"):
            size = OH
        only = os.environ.get("ONLY")  # comma list of layer-name prefixes (A/B runs)
        if only and not name.startswith(tuple(only.split(","))):
            continue
        x = torch.randn(N, H, H, cin, device=dev).to(BF16)
        w = (torch.randn(cout, CN.kpad(k, k, cin), device=dev) * 0.05).to(BF16)
        dy = torch.randn(N, OH, OW, cout, device=dev).to(BF16)
        cs = torch.zeros(cout, device=dev)
        cq = torch.zeros(cout, device=dev)
        dw = torch.zeros(cout, w.shape[1], device=dev)
        M = N * OH * OW
        flops = 2.0 * M * cout * k * k * cin
        fused_bn = name != "conv1" and not name.endswith("downsample")
        mean = torch.zeros(cin, device=dev)
        rstd = torch.ones(cin, device=dev)
        bn = (x, x, mean, rstd, torch.zeros(cin, device=dev), torch.zeros(cin, device=dev)) \
            if fused_bn else None
        xin = x.numel() * 2
        yout = dy.numel() * 2
        passes = {
            "fwd": (lambda: CN.conv_fwd(x, w, k, k, s, p, colsum=cs, colsq=cq),
                    xin + yout + w.numel() * 2),
            "dgrad": (lambda: CN.conv_dgrad(dy, w, x.shape, k, k, s, p, bn=bn),
                      yout + xin * (3 if fused_bn else 1) + w.numel() * 2),
            "wgrad": (lambda: CN.conv_wgrad(dy, x, dw, k, k, s, p), yout + xin + dw.numel() * 8),
        }
        for kind, (fn, nbytes) in passes.items():
            if name == "conv1" and kind == "dgrad":
                continue  # the model never needs the image gradient
            us = timed(fn, a.reps)
            bound = max(flops / PEAK_FLOPS, nbytes / PEAK_BW) * 1e6
            tot[kind] += us
            tot["bound"] += bound
            print(json.dumps({"layer": name, "pass": kind, "M": M, "N": cout, "K": k * k * cin,
                              "us": round(us, 1), "tflops": round(flops / us / 1e6, 1),
                              "gbs": round(nbytes / us / 1e3), "bound_us": round(bound, 1),
                              "of_bound": round(bound / us, 3)}), flush=True)
        del x, w, dy, dw
    tot = {k: round(v / 1e3, 3) for k, v in tot.items()}
    print(json.dumps({"total_ms": tot}), flush=True)


if __name__ == "__main__":
    main()
