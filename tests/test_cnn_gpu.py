"""CNN kernels (implicit-GEMM convs, BatchNorm, pooling, SGD) vs the f32 PyTorch reference."""
import pytest
import torch

from distributedtensorflowexample_amd.ops import cnn

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def _r(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) * scale


CONVS = [  # N, H, W, C, Cout, k, stride, pad
    (2, 14, 14, 64, 64, 3, 1, 1),
    (2, 14, 14, 64, 128, 3, 2, 1),
    (2, 14, 14, 64, 256, 1, 2, 0),
    (2, 9, 11, 256, 64, 1, 1, 0),
    (2, 32, 32, 8, 64, 7, 2, 3),     # the stem kernel (stem_conv.hip): one 16x16 output image
    (3, 48, 64, 8, 64, 7, 2, 3),     # stem kernel, 3 x 2 x 3 tiles per image and batch
    (2, 8, 56, 64, 64, 3, 1, 1),     # the 64-channel 3x3 kernel (conv3x3_c64.hip), 4 tiles
    (3, 16, 28, 64, 64, 3, 1, 1),    # same, 6 tiles of 8 x 28 (two tile rows per image)
    (2, 28, 28, 128, 128, 3, 1, 1),  # the 128-channel 3x3 kernel (conv3x3_c128.hip), 14 tiles
    (2, 15, 13, 64, 128, 3, 2, 1),   # stride-2 dgrad: phase classes of unequal size
    (2, 14, 14, 64, 64, 3, 2, 1),    # stride-2 dgrad on the 256x64 tile
    (2, 13, 15, 128, 64, 1, 2, 0),   # 1x1 stride 2: three of four classes have no taps
    (4, 64, 64, 256, 1024, 1, 1, 0),  # 1x1 stride 1, K = 256: the streaming kernel
    (3, 60, 60, 256, 1024, 1, 1, 0),  # same, M = 10800: ragged 256-row block and 64-row slab
    (3, 60, 60, 64, 1024, 3, 1, 1),  # 3x3 forward on the 8-phase gather (ragged M)
    (4, 64, 64, 1024, 256, 3, 2, 1),  # stride-2 dgrad classes on the 8-phase gather
    (2, 16, 16, 64, 256, 1, 1, 0),   # streaming 1x1 kernel (conv1x1.hip): forward K = 64
    (2, 8, 8, 128, 512, 1, 1, 0),    # forward K = 128, two column blocks
    (1, 8, 8, 64, 2048, 1, 1, 0),    # one 64-pixel tile, 8 column blocks, idle pixel blocks
    (2, 8, 8, 256, 1024, 1, 1, 0),   # forward K = 256 (one block per CU)
    (2, 8, 8, 1024, 256, 1, 1, 0),   # dgrad K = 256 -> 1024 channels
    (2, 16, 16, 256, 64, 1, 1, 0),   # dgrad K = 64 -> 256 channels
    (2, 8, 8, 512, 128, 1, 1, 0),    # dgrad K = 128 -> 512 channels (16-pixel tiles)
    (2, 8, 8, 256, 128, 1, 1, 0),    # narrow forward 256 -> 128 (the two above: 256 -> 64, 512 -> 128)
    (4, 14, 14, 256, 256, 3, 1, 1),  # few tiles, deep K: split-K fwd / dgrad + epilogue pass
    (2, 7, 7, 512, 512, 3, 1, 1),    # ResNet layer4 conv2 shape: M = 98 (ragged 64-row slab)
    (2, 7, 7, 2048, 512, 1, 1, 0),   # layer4 conv1 (1x1, K = 2048), split-K forward
    (4, 16, 16, 256, 512, 3, 1, 1),  # 3x3 weight gradient on the 8-phase tile (Cout >= 256)
    (4, 32, 32, 256, 256, 3, 2, 1),  # same, stride 2 (layer3.0's shape class)
    (8, 8, 8, 512, 512, 3, 1, 1),    # layer4 conv2 class: 8-phase wgrad, 2 x 18 tiles, split K
]


@pytest.mark.parametrize("N,H,W,C,Co,k,s,p", CONVS)
def test_conv_fwd_dgrad_wgrad(gpu, N, H, W, C, Co, k, s, p):
    x = _r(N, H, W, C, seed=1).to(BF)
    ld = cnn.kpad(k, k, C)
    w = torch.zeros(Co, ld)
    w[:, :k * k * C] = _r(Co, k * k * C, seed=2, scale=(k * k * C) ** -0.5)
    w = w.to(BF)
    cs, cq = torch.zeros(Co), torch.zeros(Co)
    csg, cqg = torch.zeros(Co, device=gpu), torch.zeros(Co, device=gpu)
    y = cnn.conv_fwd(x.to(gpu), w.to(gpu), k, k, s, p, colsum=csg, colsq=cqg)
    yr = cnn.conv_fwd(x, w, k, k, s, p, colsum=cs, colsq=cq)
    assert y.shape == yr.shape
    assert (y.cpu().float() - yr.float()).abs().max() < 3e-2 * yr.float().abs().max()
    assert torch.allclose(csg.cpu(), cs, rtol=1e-2, atol=0.5)
    assert torch.allclose(cqg.cpu(), cq, rtol=1e-2, atol=0.5)
    dy = _r(*yr.shape, seed=3).to(BF)
    if C % 8 == 0 and Co % 64 == 0 and C >= 64:
        dx = cnn.conv_dgrad(dy.to(gpu), w.to(gpu), x.shape, k, k, s, p)
        dxr = cnn.conv_dgrad(dy, w, x.shape, k, k, s, p)
        assert (dx.cpu().float() - dxr.float()).abs().max() < 3e-2 * dxr.float().abs().max()
    dw = torch.full((Co, ld), 0.5, device=gpu)
    dwr = torch.full((Co, ld), 0.5)
    cnn.conv_wgrad(dy.to(gpu), x.to(gpu), dw, k, k, s, p, beta=1.0)
    cnn.conv_wgrad(dy, x, dwr, k, k, s, p, beta=1.0)
    kk = k * k * C
    assert (dw.cpu()[:, :kk] - dwr[:, :kk]).abs().max() < 1e-2 * dwr[:, :kk].abs().max()
    assert (dw.cpu()[:, kk:] == 0.5).all()  # padded columns untouched


@pytest.mark.parametrize("N,H,W,C,Co,k,s,p,with_res", [
    (2, 14, 14, 64, 64, 3, 1, 1, True),
    (2, 14, 14, 64, 256, 1, 2, 0, False),
    (2, 9, 11, 256, 64, 1, 1, 0, True),   # M = 198: ragged last partial-statistics slab
    (2, 14, 14, 128, 128, 3, 2, 1, True),  # stride-2 phase classes, one partial block each
    (2, 15, 13, 64, 128, 3, 2, 1, True),   # unequal classes: zeroed partial rows
    (2, 13, 15, 128, 64, 1, 2, 0, True),   # empty classes: residual + mask only
    (2, 8, 56, 64, 64, 3, 1, 1, False),    # 64-channel 3x3 kernel with the fused BN backward
    (3, 16, 28, 64, 64, 3, 1, 1, False),   # same, 6 tiles
    (2, 28, 28, 128, 128, 3, 1, 1, False),  # 128-channel 3x3 kernel with the fused BN backward
    (4, 64, 64, 1024, 256, 3, 2, 1, True),  # 8-phase dgrad: per-slab BN columns, class rows
    (3, 60, 60, 1024, 256, 1, 1, 0, True),  # 8-phase 1x1 dgrad (M % 64 != 0: not streamed)
    (4, 64, 64, 1024, 256, 1, 1, 0, True),  # streaming 1x1 dgrad, K = 256, 4 column blocks
    (2, 16, 16, 256, 64, 1, 1, 0, True),   # streaming 1x1 dgrad (conv1x1.hip), K = 64
    (2, 8, 8, 512, 128, 1, 1, 0, True),    # K = 128, two column blocks
    (2, 16, 16, 256, 128, 1, 1, 0, False),  # K = 128 -> 256, no shortcut gradient
    (2, 16, 16, 64, 256, 1, 1, 0, False),  # narrow dgrad 256 -> 64 with the BN backward
    (2, 8, 8, 128, 512, 1, 1, 0, False),   # narrow dgrad 512 -> 128
    (2, 8, 8, 128, 256, 1, 1, 0, False),   # narrow dgrad 256 -> 128
    (2, 8, 8, 128, 512, 1, 1, 0, True),    # narrow shape + shortcut gradient: implicit GEMM
    (4, 14, 14, 256, 256, 3, 1, 1, True),  # split-K dgrad: BN backward in the epilogue pass
    (2, 7, 7, 512, 512, 3, 1, 1, False),   # layer4 conv2 shape, ragged last statistics slab
    (2, 7, 7, 512, 2048, 1, 1, 0, True),   # layer4 conv3 dgrad (K = 2048) + shortcut gradient
])
def test_conv_dgrad_fused_batchnorm_backward(gpu, N, H, W, C, Co, k, s, p, with_res):
    """(The last three cases take the split-K path: cnn.hip conv_splitk > 1.)"""
    """dgrad with BatchNorm backward's reductions in its epilogue (+ shortcut gradient, ReLU
    mask) and the apply-only BN kernel == dgrad, then the two-pass bn_bwd (f32 CPU path)."""
    c = _r(N, H, W, C, seed=11, scale=2).to(BF) + 0.5      # BN input (a conv output)
    M = N * H * W
    cf = c.float().reshape(M, C)
    mean_r, rstd_r = cnn.bn_finalize(cf.sum(0), (cf * cf).sum(0), M)
    gamma, beta = _r(C, seed=12) * 0.1 + 1, _r(C, seed=13) * 0.1
    y = cnn.bn_apply(c, mean_r, rstd_r, gamma, beta, None, relu=True)   # block input
    ld = cnn.kpad(k, k, C)
    w = torch.zeros(Co, ld)
    w[:, :k * k * C] = _r(Co, k * k * C, seed=14, scale=(k * k * C) ** -0.5)
    w = w.to(BF)
    OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = _r(N, OH, OW, Co, seed=15).to(BF)
    res = _r(N, H, W, C, seed=16).to(BF) if with_res else None
    # reference: unfused, CPU
    dconv = cnn.conv_dgrad(dy, w, c.shape, k, k, s, p, residual=res)
    dgr, dbr = torch.zeros(C), torch.zeros(C)
    dxr, der = cnn.bn_bwd(dconv, y, c, mean_r, rstd_r, gamma, dgr, dbr, True, True)
    # fused, GPU
    g = lambda t: None if t is None else t.to(gpu)  # noqa: E731
    dg, db = torch.zeros(C, device=gpu), torch.zeros(C, device=gpu)
    de = cnn.conv_dgrad(g(dy), g(w), c.shape, k, k, s, p, residual=g(res),
                        bn=(g(y), g(c), g(mean_r), g(rstd_r), db, dg))
    dx = cnn.bn_bwd_apply(de, g(c), g(mean_r), g(rstd_r), g(gamma), db, dg)
    scale = der.float().abs().max()
    assert (de.cpu().float() - der.float()).abs().max() < 3e-2 * scale
    assert ((de.cpu().float() == 0) == (der.float() == 0)).float().mean() > 0.995  # ReLU mask
    assert torch.allclose(db.cpu(), dbr, atol=0.05 * float(dbr.abs().max()) + 1e-2, rtol=2e-2)
    assert torch.allclose(dg.cpu(), dgr, atol=0.05 * float(dgr.abs().max()) + 1e-2, rtol=2e-2)
    assert (dx.cpu().float() - dxr.float()).abs().max() < 4e-2 * dxr.float().abs().max()


def test_batchnorm_fwd_bwd(gpu):
    N, H, W, C = 4, 7, 7, 64
    x = _r(N, H, W, C, seed=4, scale=2).to(BF) + 1
    res = _r(N, H, W, C, seed=5).to(BF)
    gamma, beta = _r(C, seed=6) * 0.1 + 1, _r(C, seed=7) * 0.1
    M = N * H * W
    s, q = x.float().reshape(M, C).sum(0), (x.float().reshape(M, C) ** 2).sum(0)
    mean, rstd = cnn.bn_finalize(s.to(gpu), q.to(gpu), M)
    mr, rr = cnn.bn_finalize(s, q, M)
    assert torch.allclose(mean.cpu(), mr, atol=1e-5) and torch.allclose(rstd.cpu(), rr, rtol=1e-4)
    y = cnn.bn_apply(x.to(gpu), mean, rstd, gamma.to(gpu), beta.to(gpu), res.to(gpu), relu=True)
    yr = cnn.bn_apply(x, mr, rr, gamma, beta, res, relu=True)
    assert (y.cpu().float() - yr.float()).abs().max() < 3e-2
    dy = _r(N, H, W, C, seed=8).to(BF)
    dg, db = torch.zeros(C, device=gpu), torch.zeros(C, device=gpu)
    dx, dres = cnn.bn_bwd(dy.to(gpu), y, x.to(gpu), mean, rstd, gamma.to(gpu), dg, db, True, True)
    dgr, dbr = torch.zeros(C), torch.zeros(C)
    dxr, dresr = cnn.bn_bwd(dy, y.cpu(), x, mr, rr, gamma, dgr, dbr, True, True)
    assert (dx.cpu().float() - dxr.float()).abs().max() < 3e-2 * dxr.float().abs().max()
    assert torch.equal(dres.cpu(), dresr)
    assert torch.allclose(dg.cpu(), dgr, atol=1e-2, rtol=1e-3)
    assert torch.allclose(db.cpu(), dbr, atol=1e-2, rtol=1e-3)


@pytest.mark.parametrize("C", [64, 96, 2048])  # 96: the general (per-element channel) path
def test_batchnorm_apply_from_sums(gpu, C):
    """Fused finalize + apply (bn_apply_stats): mean / rstd / running statistics and the output
    match bn_finalize + bn_apply on the CPU; with res_bn the residual (a raw conv output) is
    normalised by its own statistics and affine before the add."""
    N, H, W = 4, 7, 9
    M = N * H * W
    x = _r(N, H, W, C, seed=20, scale=2).to(BF) + 1
    r = _r(N, H, W, C, seed=21, scale=3).to(BF) - 0.5
    g1, b1 = _r(C, seed=22) * 0.1 + 1, _r(C, seed=23) * 0.1
    g2, b2 = _r(C, seed=24) * 0.1 + 1, _r(C, seed=25) * 0.1
    xf, rf = x.float().reshape(M, C), r.float().reshape(M, C)
    s1, q1, s2, q2 = xf.sum(0), (xf * xf).sum(0), rf.sum(0), (rf * rf).sum(0)
    # single BN, residual added as is
    rm, rv = torch.zeros(C), torch.ones(C)
    yr, mr, rr = cnn.bn_apply_stats(x, s1, q1, M, g1, b1, r, True, 1e-5, rm, rv)
    rmg, rvg = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
    y, m, rs = cnn.bn_apply_stats(x.to(gpu), s1.to(gpu), q1.to(gpu), M, g1.to(gpu), b1.to(gpu),
                                  r.to(gpu), True, 1e-5, rmg, rvg)
    assert torch.allclose(m.cpu(), mr, atol=1e-5) and torch.allclose(rs.cpu(), rr, rtol=1e-4)
    assert torch.allclose(rmg.cpu(), rm, atol=1e-5) and torch.allclose(rvg.cpu(), rv, rtol=1e-4)
    # (one bf16 ulp of outputs up to ~6)
    assert (y.cpu().float() - yr.float()).abs().max() < 1e-2 * yr.float().abs().max() + 1e-2
    # residual through its own BN (the downsample shortcut of a bottleneck)
    rm1, rv1, rm2, rv2 = torch.zeros(C), torch.ones(C), torch.zeros(C), torch.ones(C)
    yr, mr, rr, mr2, rr2 = cnn.bn_apply_stats(x, s1, q1, M, g1, b1, r, True, 1e-5, rm1, rv1,
                                              res_bn=(s2, q2, g2, b2, rm2, rv2))
    dev = [t.to(gpu) for t in (rm1.new_zeros(C), rv1.new_ones(C), rm2.new_zeros(C), rv2.new_ones(C))]
    y, m, rs, m2, r2 = cnn.bn_apply_stats(
        x.to(gpu), s1.to(gpu), q1.to(gpu), M, g1.to(gpu), b1.to(gpu), r.to(gpu), True, 1e-5, dev[0],
        dev[1], res_bn=(s2.to(gpu), q2.to(gpu), g2.to(gpu), b2.to(gpu), dev[2], dev[3]))
    for a, b in ((m, mr), (m2, mr2), (dev[0], rm1), (dev[2], rm2)):
        assert torch.allclose(a.cpu(), b, atol=1e-5)
    for a, b in ((rs, rr), (r2, rr2), (dev[1], rv1), (dev[3], rv2)):
        assert torch.allclose(a.cpu(), b, rtol=1e-4)
    # (the CPU reference rounds the normalised shortcut to bf16 before the add)
    assert (y.cpu().float() - yr.float()).abs().max() < 2e-2 * yr.float().abs().max() + 1e-2


def test_pools(gpu):
    x = _r(2, 15, 16, 64, seed=9).to(BF)
    y, idx = cnn.maxpool_fwd(x.to(gpu))
    yr, idxr = cnn.maxpool_fwd(x)
    assert torch.equal(y.cpu(), yr)
    dy = _r(*yr.shape, seed=10).to(BF)
    dx = cnn.maxpool_bwd(dy.to(gpu), idx, x.shape)
    dxr = cnn.maxpool_bwd(dy, idxr, x.shape)
    assert (dx.cpu().float() - dxr.float()).abs().max() < 2e-2
    a = cnn.avgpool_fwd(x.to(gpu))
    assert (a.cpu().float() - cnn.avgpool_fwd(x).float()).abs().max() < 1e-2
    da = _r(2, 64, seed=11).to(BF)
    assert (cnn.avgpool_bwd(da.to(gpu), x.shape).cpu().float() -
            cnn.avgpool_bwd(da, x.shape).float()).abs().max() < 1e-3


def test_sgd_momentum_mixed(gpu):
    p, g = _r(1024, seed=12), _r(1024, seed=13)
    v = torch.zeros(1024)
    P, G, V = p.to(gpu), g.to(gpu), v.to(gpu)
    pb = torch.empty(1024, device=gpu, dtype=BF)
    for _ in range(3):
        cnn.sgd_momentum_mixed(P, G, V, pb, 0.1, 0.9, 1e-4, 0.5)
        cnn.sgd_momentum_mixed(p, g, v, None, 0.1, 0.9, 1e-4, 0.5)
    assert torch.allclose(P.cpu(), p, atol=1e-6)
    assert torch.equal(pb.cpu(), P.cpu().to(BF))


@pytest.mark.parametrize("N,H,W,C,Co", [(2, 16, 16, 256, 64), (2, 8, 8, 512, 128),
                                         (2, 8, 8, 1024, 256)])
def test_conv1x1_dgrad_residual_only(gpu, N, H, W, C, Co):
    """The first bottleneck's conv1 dgrad: the shortcut gradient added, no BN fused."""
    w = _r(Co, C, seed=21, scale=C ** -0.5).to(BF)
    dy = _r(N, H, W, Co, seed=22).to(BF)
    res = _r(N, H, W, C, seed=23).to(BF)
    dx = cnn.conv_dgrad(dy.to(gpu), w.to(gpu), (N, H, W, C), 1, 1, 1, 0, residual=res.to(gpu))
    dxr = cnn.conv_dgrad(dy, w, (N, H, W, C), 1, 1, 1, 0, residual=res)
    assert (dx.cpu().float() - dxr.float()).abs().max() < 3e-2 * dxr.float().abs().max()


@pytest.mark.parametrize("N,H,W,K,Co,ds", [
    (2, 16, 16, 256, 64, False),   # layer1 block output -> next conv1 (256 -> 64)
    (2, 16, 16, 256, 64, True),    # first block: shortcut through the downsample BN
    (4, 8, 8, 256, 128, True),     # layer1 -> layer2.0 conv1 (256 -> 128)
    (4, 8, 8, 512, 128, False),    # layer2 block output -> next conv1 (512 -> 128), 16-pixel tiles
    (3, 16, 20, 512, 128, True),   # M = 960: tiles spread unevenly over the 256 blocks
])
def test_bn_out_conv1x1_prologue(gpu, N, H, W, K, Co, ds):
    """The bottleneck output relu(bn3(c3) + shortcut) formed inside the next 1x1 conv's prologue
    (conv1x1.hip PRO 1) == bn_apply_stats then conv_fwd (f32 CPU path): the block output, the
    conv output, its statistics, mean / rstd and the running statistics."""
    M = N * H * W
    c = _r(N, H, W, K, seed=31, scale=2).to(BF) + 0.5
    r = _r(N, H, W, K, seed=32, scale=1.5).to(BF) - 0.25
    g1, b1 = _r(K, seed=33) * 0.1 + 1, _r(K, seed=34) * 0.1
    g2, b2 = _r(K, seed=35) * 0.1 + 1, _r(K, seed=36) * 0.1
    cf, rf = c.float().reshape(M, K), r.float().reshape(M, K)
    s, q, s2, q2 = cf.sum(0), (cf * cf).sum(0), rf.sum(0), (rf * rf).sum(0)
    w = _r(Co, K, seed=37, scale=K ** -0.5).to(BF)

    def run(dev):
        t = lambda v: v.to(dev)  # noqa: E731
        cs, cq = torch.zeros(Co, device=dev), torch.zeros(Co, device=dev)
        run_st = [torch.zeros(K, device=dev), torch.ones(K, device=dev),
                  torch.zeros(K, device=dev), torch.ones(K, device=dev)]
        res_bn = (t(s2), t(q2), t(g2), t(b2), run_st[2], run_st[3]) if ds else None
        out = cnn.bn_out_conv1x1(t(c), t(s), t(q), M, t(g1), t(b1), t(r), t(w), cs, cq, 1e-5,
                                 run_st[0], run_st[1], res_bn=res_bn)
        return [v.cpu() for v in out] + [cs.cpu(), cq.cpu()] + [v.cpu() for v in run_st]

    got, ref = run(gpu), run("cpu")
    assert len(got) == len(ref) == (12 if ds else 10)
    o, orf = got[0].float(), ref[0].float()
    # (the CPU reference rounds the normalised shortcut to bf16 before the add)
    assert (o - orf).abs().max() < 2e-2 * orf.abs().max() + 1e-2
    assert ((o == 0) == (orf == 0)).float().mean() > 0.995          # ReLU
    y, yr = got[1].float(), ref[1].float()
    assert (y - yr).abs().max() < 3e-2 * yr.abs().max()
    for a, b in zip(got[2:], ref[2:]):  # mean / rstd (x2), column sums, running statistics
        assert torch.allclose(a, b, rtol=2e-2, atol=1e-2 * float(b.abs().max()) + 1e-4)
    # the GPU prologue against the GPU's own two-pass path: the same block output
    rb = (s2.to(gpu), q2.to(gpu), g2.to(gpu), b2.to(gpu), None, None) if ds else None
    two = cnn.bn_apply_stats(c.to(gpu), s.to(gpu), q.to(gpu), M, g1.to(gpu), b1.to(gpu),
                             r.to(gpu), True, 1e-5, res_bn=rb)
    d = (two[0].cpu().float() - o).abs()
    assert (d <= 2 ** -7 * o.abs() + 1e-6).all()  # at most one bf16 rounding apart


@pytest.mark.parametrize("N,H,W,Cin,K,with_res,with_bn", [
    (2, 16, 16, 64, 256, False, True),    # layer1 conv3 data gradient (narrow 256 -> 64)
    (4, 8, 8, 128, 512, False, True),     # layer2 conv3 (narrow 512 -> 128, 16-pixel tiles)
    (3, 16, 20, 64, 256, False, True),    # M = 960
    (2, 16, 16, 64, 256, False, False),   # layer1.0 downsample (narrow, plain: PRO 4)
    (4, 8, 8, 128, 512, False, False),    # narrow 512 -> 128 plain
    (2, 16, 16, 256, 64, True, True),     # layer1 conv1 (wide 64 -> 256, + shortcut gradient)
    (2, 16, 16, 256, 64, True, False),    # first block's conv1: shortcut only, no BN behind
    (2, 8, 8, 512, 128, True, True),      # layer2 conv1 (two column blocks: xo from one)
    (2, 8, 8, 1024, 256, True, True),     # layer3 conv1 (four column blocks)
])
def test_bn_in_conv1x1_dgrad_prologue(gpu, N, H, W, Cin, K, with_res, with_bn):
    """A BatchNorm's backward apply formed inside the dgrad prologue of the 1x1 conv feeding it
    (conv1x1.hip PRO 2: narrow conv3 / wide conv1 products) == bn_bwd_apply then the dgrad with
    the fused BN reductions of the conv's own input and the shortcut gradient (f32 CPU path):
    dL/dc (written for the weight gradient), the dgrad output and the input BN's sums."""
    M = N * H * W
    c3 = _r(N, H, W, K, seed=41, scale=2).to(BF) + 0.5
    c3f = c3.float().reshape(M, K)
    m3, r3 = cnn.bn_finalize(c3f.sum(0), (c3f * c3f).sum(0), M)
    g3 = _r(K, seed=42) * 0.1 + 1
    de3 = _r(N, H, W, K, seed=43).to(BF)
    d3 = de3.float().reshape(M, K)
    sdy3, sdx3 = d3.sum(0), (d3 * (c3f - m3) * r3).sum(0)
    c2 = _r(N, H, W, Cin, seed=44, scale=2).to(BF) + 0.5
    c2f = c2.float().reshape(M, Cin)
    m2, r2 = cnn.bn_finalize(c2f.sum(0), (c2f * c2f).sum(0), M)
    g2, b2 = _r(Cin, seed=45) * 0.1 + 1, _r(Cin, seed=46) * 0.1
    y2 = cnn.bn_apply(c2, m2, r2, g2, b2, None, relu=True)
    w3 = _r(K, Cin, seed=47, scale=Cin ** -0.5).to(BF)
    res = _r(N, H, W, Cin, seed=48).to(BF) if with_res else None

    def run(dev):
        t = lambda v: None if v is None else v.to(dev)  # noqa: E731
        sdy2, sdx2 = torch.zeros(Cin, device=dev), torch.zeros(Cin, device=dev)
        bn = (t(y2), t(c2), t(m2), t(r2), sdy2, sdx2) if with_bn else None
        dx, dc = cnn.bn_in_conv1x1_dgrad(t(de3), t(c3), t(m3), t(r3), t(g3), t(sdy3), t(sdx3),
                                         t(w3), bn, residual=t(res))
        return dx.cpu().float(), dc.cpu().float(), sdy2.cpu(), sdx2.cpu()

    (dx, dc, a, b), (dxr, dcr, ar, br) = run(gpu), run("cpu")
    assert (dc - dcr).abs().max() < 2e-2 * dcr.abs().max()
    assert (dx - dxr).abs().max() < 3e-2 * dxr.abs().max()
    if not with_bn:
        return
    assert ((dx == 0) == (dxr == 0)).float().mean() > 0.995    # the input BN's ReLU mask
    assert torch.allclose(a, ar, atol=0.05 * float(ar.abs().max()) + 1e-2, rtol=2e-2)
    assert torch.allclose(b, br, atol=0.05 * float(br.abs().max()) + 1e-2, rtol=2e-2)


@pytest.mark.parametrize("N,H,W,Cin,K", [
    (2, 16, 16, 256, 128),   # layer2.0 conv1's data gradient + the downsample's (56 -> 28)
    (2, 6, 16, 512, 256),    # layer3.0 class (two column blocks; a tile spans two grid rows)
])
def test_bn_in_conv1x1_dgrad_compact_residual(gpu, N, H, W, Cin, K):
    """A stride-2 1x1 conv's data gradient kept compact [N, H/2, W/2, Cin] and read by the
    wide dgrad kernel as a residual that is zero at odd rows / columns (conv1x1.hip rs_h /
    rs_w) == the same residual expanded to full resolution (f32 CPU path)."""
    M = N * H * W
    c1 = _r(N, H, W, K, seed=61, scale=2).to(BF) + 0.5
    c1f = c1.float().reshape(M, K)
    m1, r1 = cnn.bn_finalize(c1f.sum(0), (c1f * c1f).sum(0), M)
    g1 = _r(K, seed=62) * 0.1 + 1
    de1 = _r(N, H, W, K, seed=63).to(BF)
    d1 = de1.float().reshape(M, K)
    sdy1, sdx1 = d1.sum(0), (d1 * (c1f - m1) * r1).sum(0)
    cx = _r(N, H, W, Cin, seed=64, scale=2).to(BF) + 0.5
    cxf = cx.float().reshape(M, Cin)
    mx, rx = cnn.bn_finalize(cxf.sum(0), (cxf * cxf).sum(0), M)
    yx = cnn.bn_apply(cx, mx, rx, _r(Cin, seed=65) * 0.1 + 1, _r(Cin, seed=66) * 0.1, None,
                      relu=True)
    w1 = _r(K, Cin, seed=67, scale=Cin ** -0.5).to(BF)
    rc = _r(N, H // 2, W // 2, Cin, seed=68).to(BF)
    full = torch.zeros(N, H, W, Cin, dtype=BF)
    full[:, ::2, ::2] = rc

    def run(dev, res, s2):
        t = lambda v: v.to(dev)  # noqa: E731
        sdy, sdx = torch.zeros(Cin, device=dev), torch.zeros(Cin, device=dev)
        dx, _ = cnn.bn_in_conv1x1_dgrad(t(de1), t(c1), t(m1), t(r1), t(g1), t(sdy1), t(sdx1),
                                        t(w1), (t(yx), t(cx), t(mx), t(rx), sdy, sdx),
                                        residual=t(res), residual_s2=s2)
        return dx.cpu().float(), sdy.cpu(), sdx.cpu()

    dx, a, b = run(gpu, rc, True)
    dxr, ar, br = run("cpu", full, False)
    assert (dx - dxr).abs().max() < 3e-2 * dxr.abs().max()
    assert torch.allclose(a, ar, atol=0.05 * float(ar.abs().max()) + 1e-2, rtol=2e-2)
    assert torch.allclose(b, br, atol=0.05 * float(br.abs().max()) + 1e-2, rtol=2e-2)
    dxg, _, _ = run(gpu, full, False)   # the full-resolution residual on the same kernel
    assert (dx - dxg).abs().max() <= 1e-6 + 2 ** -7 * dxg.abs().max()


@pytest.mark.parametrize("N,H,W", [(2, 8, 56), (3, 16, 28)])
def test_bn_relu_conv3x3_c64_prologue(gpu, N, H, W):
    """relu(bn(c)) formed in the 64-channel 3x3 kernel's patch staging (conv3x3_c64.hip PRO),
    written once to a, then the conv with its output statistics == bn_apply_stats then conv_fwd
    (f32 CPU path): a, y, the column sums, mean / rstd and the running statistics."""
    C = 64
    M = N * H * W
    c = _r(N, H, W, C, seed=71, scale=2).to(BF) + 0.25
    cf = c.float().reshape(M, C)
    s, q = cf.sum(0), (cf * cf).sum(0)
    g, b = _r(C, seed=72) * 0.1 + 1, _r(C, seed=73) * 0.1
    w = (_r(C, 9 * C, seed=74, scale=(9 * C) ** -0.5)).to(BF)

    def run(dev):
        t = lambda v: v.to(dev)  # noqa: E731
        cs, cq = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        a, y, m, r = cnn.bn_relu_conv3x3(t(c), t(s), t(q), M, t(g), t(b), t(w), cs, cq, 1e-5,
                                         rm, rv)
        return [v.cpu().float() for v in (a, y, cs, cq, m, r, rm, rv)]

    got, ref = run(gpu), run("cpu")
    a, y = got[0], got[1]
    assert (a - ref[0]).abs().max() <= 2 ** -7 * ref[0].abs().max() + 1e-6
    assert (y - ref[1]).abs().max() < 3e-2 * ref[1].abs().max()
    for x_, r_ in zip(got[2:], ref[2:]):
        assert torch.allclose(x_, r_, rtol=1e-2, atol=1e-2 * float(r_.abs().max()) + 1e-5)


@pytest.mark.parametrize("N,H,W", [(2, 16, 16), (3, 15, 17)])   # odd sizes: clipped windows
def test_stem_bn_maxpool_fused(gpu, N, H, W):
    """The stem's maxpool(relu(bn(c))) with relu(bn(c)) never stored (maxpool_bn_fwd_kernel) and
    its two-pass backward (re-gathered pool gradient: BatchNorm sums, then the apply) == the
    separate bn_apply_stats / maxpool / maxpool_bwd / bn_bwd passes (f32 CPU path)."""
    C = 64
    M = N * H * W
    c = _r(N, H, W, C, seed=51, scale=2).to(BF) + 0.25
    cf = c.float().reshape(M, C)
    s, q = cf.sum(0), (cf * cf).sum(0)
    g, b = _r(C, seed=52) * 0.1 + 1, _r(C, seed=53) * 0.1

    def run(dev, idx_bwd=None):
        t = lambda v: v.to(dev)  # noqa: E731
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        y, idx, m, r, fco = cnn.bn_maxpool_fwd(t(c), t(s), t(q), M, t(g), t(b), 1e-5, rm, rv)
        if idx_bwd is not None:  # the backward of both paths routes through the same taps
            idx = t(idx_bwd)
        dy = _r(*y.shape, seed=54).to(BF).to(dev)
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        dc = cnn.maxpool_bn_bwd(dy, idx, t(c), m, r, t(g), t(b), fco, dg, db)
        return [v.cpu() for v in (y, idx, m, r, rm, rv, dc, dg, db)]

    (y, idx, m, r, rm, rv, dc, dg, db) = run(gpu)
    (yr, idxr, mr, rr, rmr, rvr, dcr, dgr, dbr) = run("cpu", idx)
    # (same bf16 activations inside every window: identical maxima and argmax taps, bar ties
    # created by one-ulp differences in the normalisation)
    assert (y.float() - yr.float()).abs().max() < 1e-2 * yr.float().abs().max() + 1e-2
    yr2, idxr2 = cnn.maxpool_fwd(cnn.bn_apply(c, mr, rr, g, b, None, relu=True))
    assert (idx == idxr2).float().mean() > 0.99
    for a_, b_ in ((m, mr), (rm, rmr)):
        assert torch.allclose(a_, b_, atol=1e-5)
    for a_, b_ in ((r, rr), (rv, rvr)):
        assert torch.allclose(a_, b_, rtol=1e-4)
    assert (dc.float() - dcr.float()).abs().max() < 4e-2 * dcr.float().abs().max()
    assert torch.allclose(db, dbr, atol=0.05 * float(dbr.abs().max()) + 1e-2, rtol=2e-2)
    assert torch.allclose(dg, dgr, atol=0.05 * float(dgr.abs().max()) + 1e-2, rtol=2e-2)


@pytest.mark.parametrize("N,H,W,K,Co", [
    (2, 16, 16, 64, 256),     # layer1 conv2 BN -> conv3 (64 -> 256)
    (2, 8, 8, 128, 512),      # layer2 (two column blocks: a written by one)
    (2, 8, 8, 256, 1024),     # layer3 (four column blocks, one block per CU)
    (3, 16, 20, 64, 256),     # M = 960: ragged tiles over the persistent blocks
])
def test_bn_relu_conv1x1_prologue(gpu, N, H, W, K, Co):
    """relu(bn(c)) formed inside the wide 1x1 forward kernel's prologue (conv1x1.hip PRO 3) and
    written once == bn_apply_stats then conv_fwd (f32 CPU path)."""
    M = N * H * W
    c = _r(N, H, W, K, seed=61, scale=2).to(BF) + 0.5
    cf = c.float().reshape(M, K)
    s_, q_ = cf.sum(0), (cf * cf).sum(0)
    g, b = _r(K, seed=62) * 0.1 + 1, _r(K, seed=63) * 0.1
    w = _r(Co, K, seed=64, scale=K ** -0.5).to(BF)

    def run(dev):
        t = lambda v: v.to(dev)  # noqa: E731
        cs, cq = torch.zeros(Co, device=dev), torch.zeros(Co, device=dev)
        rm, rv = torch.zeros(K, device=dev), torch.ones(K, device=dev)
        a, y, m, r = cnn.bn_relu_conv1x1(t(c), t(s_), t(q_), M, t(g), t(b), t(w), cs, cq, 1e-5, rm, rv)
        return [v.cpu() for v in (a, y, m, r, cs, cq, rm, rv)]

    got, ref = run(gpu), run("cpu")
    a, ar = got[0].float(), ref[0].float()
    d = (a - ar).abs()
    assert (d <= 2 ** -7 * ar.abs() + 1e-6).all()  # at most one bf16 rounding apart
    assert (got[1].float() - ref[1].float()).abs().max() < 3e-2 * ref[1].float().abs().max()
    for x_, y_ in zip(got[2:], ref[2:]):
        assert torch.allclose(x_, y_, rtol=2e-2, atol=1e-2 * float(y_.abs().max()) + 1e-4)


def test_stem_wgrad_bn_prologue(gpu):
    """The stem weight gradient forming dL/dc = bn_bwd_apply(de, c) as it stages its dy tile
    (stem_conv_wgrad_kernel<true>, coefficients from maxpool_bn_bwd(apply=False)) == the apply
    pass then the plain stem weight gradient."""
    N, H, W = 2, 32, 32   # stem: 7x7 / 2 -> 16 x 16, 64 channels
    img = _r(N, H, W, 8, seed=71).to(BF)
    img[..., 3:] = 0
    w = torch.zeros(64, cnn.kpad(7, 7, 8))
    w[:, :392] = _r(64, 392, seed=72, scale=392 ** -0.5)
    w = w.to(BF)
    g_ = lambda t: t.to(gpu)  # noqa: E731
    C = 64
    cs, cq = torch.zeros(C, device=gpu), torch.zeros(C, device=gpu)
    c = cnn.conv_fwd(g_(img), g_(w), 7, 7, 2, 3, colsum=cs, colsq=cq)
    M = c.numel() // C
    gam, bet = g_(_r(C, seed=73) * 0.1 + 1), g_(_r(C, seed=74) * 0.1)
    y, idx, m, r, fco = cnn.bn_maxpool_fwd(c, cs, cq, M, gam, bet)
    dy = g_(_r(*y.shape, seed=75).to(BF))
    dg1, db1 = torch.zeros(C, device=gpu), torch.zeros(C, device=gpu)
    dg2, db2 = torch.zeros(C, device=gpu), torch.zeros(C, device=gpu)
    dc = cnn.maxpool_bn_bwd(dy, idx, c, m, r, gam, bet, fco, dg1, db1)
    ref = torch.zeros(64, w.shape[1], device=gpu)
    cnn.conv_wgrad(dc, g_(img), ref, 7, 7, 2, 3, beta=1.0)
    de, bco = cnn.maxpool_bn_bwd(dy, idx, c, m, r, gam, bet, fco, dg2, db2, apply=False)
    got = torch.zeros(64, w.shape[1], device=gpu)
    assert cnn.stem_wgrad_bn_applies(g_(img), 64, 7, 2, 3)
    cnn.conv_wgrad(de, g_(img), got, 7, 7, 2, 3, beta=1.0, bn_in=(c, bco))
    assert torch.allclose(dg1, dg2) and torch.allclose(db1, db2)
    # (both form the same bf16 dc; the f32 atomics sum in different orders)
    assert (got - ref).abs().max() < 1e-3 * ref.abs().max()


@pytest.mark.parametrize("N,H,W,K,Co,ds", [
    (2, 16, 16, 256, 64, True),    # narrow forward (PRO 1) with the downsample's own BN
    (4, 8, 8, 512, 128, False),    # narrow forward, identity shortcut
])
def test_bn_coefficients_formed_in_kernel_match_coef_launch(gpu, monkeypatch, N, H, W, K, Co, ds):
    """the 1x1 prologue kernels form the BatchNorm coefficients themselves
    (bn_common.h BnCoefSrc; block 0 writes mean / rstd / running statistics) instead of reading
    the rows of a bn_fwd_coef / bn_bwd_coef launch.  Against that separate launch on the GPU:
    the same outputs and statistics for the three prologue forms (bottleneck output -> narrow
    conv1, BN + ReLU -> wide expansion, BN backward -> data gradients) -- at most one f32
    rounding apart in the coefficients (the compiler may contract them differently)."""
    M = N * H * W
    c = (_r(N, H, W, K, seed=71, scale=2) + 0.5).to(BF).to(gpu)
    r = (_r(N, H, W, K, seed=72, scale=1.5) - 0.25).to(BF).to(gpu)
    cf, rf = c.float().reshape(M, K), r.float().reshape(M, K)
    s, q, s2, q2 = cf.sum(0), (cf * cf).sum(0), rf.sum(0), (rf * rf).sum(0)
    g1, b1 = (_r(K, seed=73) * 0.1 + 1).to(gpu), (_r(K, seed=74) * 0.1).to(gpu)
    g2, b2 = (_r(K, seed=75) * 0.1 + 1).to(gpu), (_r(K, seed=76) * 0.1).to(gpu)
    w = _r(Co, K, seed=77, scale=K ** -0.5).to(BF).to(gpu)
    w_exp = _r(4 * Co, Co, seed=78, scale=Co ** -0.5).to(BF).to(gpu)
    ys = (_r(N, H, W, Co, seed=82, scale=2) + 0.3).to(BF).to(gpu)
    ysf = ys.float().reshape(M, Co)
    ys_s, ys_q = ysf.sum(0), (ysf * ysf).sum(0)

    def close(a, b, name):
        bf = a.dtype == BF
        a, b = a.float(), b.float()
        d = (a - b).abs()
        tol = (2 ** -7 * b.abs() + 1e-6) if bf else (1e-5 * b.abs().max() + 1e-7)
        assert (d <= tol).all(), (name, d.max().item())

    outs = {}
    for fused in (True, False):
        monkeypatch.setattr(cnn, "_BN_COEF_FUSED", fused)
        res = {}
        cs, cq = torch.zeros(Co, device=gpu), torch.zeros(Co, device=gpu)
        rs = [torch.zeros(K, device=gpu), torch.ones(K, device=gpu),
              torch.zeros(K, device=gpu), torch.ones(K, device=gpu)]
        rb = (s2, q2, g2, b2, rs[2], rs[3]) if ds else None
        o = cnn.bn_out_conv1x1(c, s, q, M, g1, b1, r, w, cs, cq, 1e-5, rs[0], rs[1], res_bn=rb)
        res["out"] = list(o) + [cs, cq] + rs
        # BN + ReLU of a Co-channel tensor inside the expansion (PRO 3), fixed inputs
        ycs, ycq = torch.zeros(4 * Co, device=gpu), torch.zeros(4 * Co, device=gpu)
        rm, rv = torch.zeros(Co, device=gpu), torch.ones(Co, device=gpu)
        e = cnn.bn_relu_conv1x1(ys, ys_s, ys_q, M, g1[:Co].contiguous(), b1[:Co].contiguous(),
                                w_exp, ycs, ycq, 1e-5, rm, rv)
        res["exp"] = list(e) + [ycs, ycq, rm, rv]
        # BN backward's apply inside the narrow data gradient of the K-output conv that
        # produced c (PRO 2, with the fused BN reductions of that conv's Co-channel input)
        de = (_r(N, H, W, K, seed=79)).to(BF).to(gpu)
        m3, r3 = res["out"][2], res["out"][3]
        dd = de.float().reshape(M, K)
        sdy, sdx = dd.sum(0), (dd * (cf - m3) * r3).sum(0)
        c2 = (_r(N, H, W, Co, seed=80, scale=2) + 0.5).to(BF).to(gpu)
        c2f = c2.float().reshape(M, Co)
        m2, r2 = cnn.bn_finalize(c2f.sum(0), (c2f * c2f).sum(0), M)
        y2 = cnn.bn_apply(c2, m2, r2, g2[:Co].contiguous(), b2[:Co].contiguous(), None, relu=True)
        w3 = _r(K, Co, seed=81, scale=Co ** -0.5).to(BF).to(gpu)
        sd2, sx2 = torch.zeros(Co, device=gpu), torch.zeros(Co, device=gpu)
        dx, dc = cnn.bn_in_conv1x1_dgrad(de, c, m3, r3, g1, sdy, sdx, w3,
                                         (y2, c2, m2, r2, sd2, sx2))
        res["bwd"] = [dx, dc, sd2, sx2]
        outs[fused] = res
    for key in ("out", "exp", "bwd"):
        for i, (a, b) in enumerate(zip(outs[True][key], outs[False][key])):
            close(a, b, "%s[%d]" % (key, i))
