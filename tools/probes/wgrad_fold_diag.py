import torch, sys
sys.path.insert(0, '.')
from distributedtensorflowexample_amd.ops import cnn as CN
dev = torch.device('cuda:0')
torch.manual_seed(0)
for (N, H, W, C, Cout, k, s, p) in [(32, 28, 28, 256, 512, 1, 2, 0), (32, 28, 28, 64, 64, 3, 1, 1),
                                    (32, 28, 28, 64, 256, 1, 1, 0), (32, 14, 14, 128, 128, 3, 1, 1)]:
    OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    dy = torch.randn(N, OH, OW, Cout, device=dev).to(torch.bfloat16)
    ldw = k * k * C
    dw = torch.zeros(Cout, ldw, device=dev)
    CN.conv_wgrad(dy, x, dw, k, k, s, p, beta=1.0)
    n = CN.wgrad_fold_planes(tuple(x.shape), Cout, k, k, s, p, ldw)
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (Cout, C, k, k), dy.float().permute(0, 3, 1, 2), stride=s, padding=p).permute(0, 2, 3, 1).reshape(Cout, -1)
    line = "shape %s: reduce err %.3e" % ((N, H, W, C, Cout, k, s, p), ((dw - ref).abs().max() / ref.abs().max()).item())
    if n:
        planes = torch.zeros(n, device=dev)
        dw2 = torch.zeros(Cout, ldw, device=dev)
        CN.conv_wgrad(dy, x, dw2, k, k, s, p, beta=1.0, planes=planes)
        S = n // (Cout * ldw)
        g = planes.view(S, Cout, ldw).sum(0)
        line += " | fold S=%d err %.3e, dw untouched %s" % (S, ((g - ref).abs().max() / ref.abs().max()).item(), bool((dw2 == 0).all()))
    print(line, flush=True)
