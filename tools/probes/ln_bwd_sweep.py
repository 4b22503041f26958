"""LayerNorm backward at the BERT-base shape (T = 16384, H = 768, residual + bias-grad
column sums fused), one JSON line.  Sweep rows per block with DTFX_LN_RPB=<n>."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from distributedtensorflowexample_amd.ops import transformer as TR  # noqa: E402
from tools.gemm_bench import timeit  # noqa: E402

dev = torch.device("cuda:0")
T, H = 16384, 768
x = torch.randn(T, H, device=dev).to(torch.bfloat16)
dy = torch.randn(T, H, device=dev).to(torch.bfloat16)
dres = torch.randn(T, H, device=dev).to(torch.bfloat16)
g, b = torch.ones(H, device=dev), torch.zeros(H, device=dev)
_, mean, rstd = TR.layernorm_fwd(x, g, b)
dg, db, ds = (torch.zeros(H, device=dev) for _ in range(3))
t = timeit(lambda: TR.layernorm_bwd(dy, x, mean, rstd, g, dg, db, dres=dres, dxsum=ds), iters=50)
# correctness vs the f32 CPU path
dg.zero_(); db.zero_(); ds.zero_()
dx = TR.layernorm_bwd(dy, x, mean, rstd, g, dg, db, dres=dres, dxsum=ds)
dgc, dbc, dsc = torch.zeros(H), torch.zeros(H), torch.zeros(H)
dxc = TR.layernorm_bwd(dy.cpu(), x.cpu(), mean.cpu(), rstd.cpu(), g.cpu(), dgc, dbc, dres=dres.cpu(),
                       dxsum=dsc)
err = float((dx.cpu().float() - dxc.float()).abs().max())
gerr = float(max((dg.cpu() - dgc).abs().max(), (db.cpu() - dbc).abs().max(), (ds.cpu() - dsc).abs().max()))
print(json.dumps({"rpb": os.environ.get("DTFX_LN_RPB", "default"), "us": round(t * 1e6, 2),
                  "GBps": round(T * H * 8 / t / 1e9), "dx_err": err, "param_err": gerr}))
