"""Time the compact stride-2 downsample data gradient (a 1x1 stride-1 product on the
subsampled grid) on the conv path and as a plain GEMM with each tile configuration, at the
ResNet-50 batch-256 shapes (layer2.0: 200704 x 256 x 512, layer3.0: 50176 x 512 x 1024)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from distributedtensorflowexample_amd.ops import bf16 as B16  # noqa: E402
from distributedtensorflowexample_amd.ops import cnn  # noqa: E402
from distributedtensorflowexample_amd.ops._ext import hip  # noqa: E402


def t(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / reps


for name, (n, h, w, cin, cout) in {"layer2.0": (256, 28, 28, 256, 512),
                                   "layer3.0": (256, 14, 14, 512, 1024)}.items():
    dcs = torch.randn(n, h, w, cout, device="cuda").to(torch.bfloat16)
    wt = (torch.randn(cout, cin, device="cuda") * cout ** -0.5).to(torch.bfloat16)
    r = {"layer": name, "M": n * h * w, "N": cin, "K": cout}
    r["conv_dgrad_us"] = round(t(lambda: cnn.conv_dgrad(dcs, wt, (n, h, w, cin), 1, 1, 1, 0)), 1)
    a2 = dcs.view(-1, cout)
    ref = None
    for cfg in (-1, 0, 5, 6):
        hip().gemm_bf16_set_cfg(cfg)
        r["gemm_cfg%d_us" % cfg] = round(t(lambda: B16.gemm(a2, wt)), 1)
        o = B16.gemm(a2, wt).float()
        ref = o if ref is None else ref
        r["gemm_cfg%d_err" % cfg] = float((o - ref).abs().max())
    hip().gemm_bf16_set_cfg(-1)
    print(json.dumps(r), flush=True)
