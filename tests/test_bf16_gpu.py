"""bf16 matrix-core kernels vs an f32 PyTorch reference of the same op (1 GPU)."""
import pytest
import torch

from distributedtensorflowexample_amd.ops import bf16

pytestmark = pytest.mark.gpu


def _rand(*shape, dev, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return ((torch.rand(*shape, generator=g) * 2 - 1) * scale).to(dev).to(torch.bfloat16)


def _ref(a, b, ta, tb):
    A = a.float().t() if ta else a.float()
    B = b.float().t() if tb else b.float()
    return A @ B


@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False), (True, True)])
def test_gemm_exact_integers(gpu, ta, tb):
    # small integers: every product and partial sum is exact in f32, so any
    # layout / fragment-map / swizzle error shows as an exact mismatch.
    M, N, K = 256, 384, 192
    g = torch.Generator().manual_seed(7)
    a = torch.randint(-4, 5, ((K, M) if ta else (M, K)), generator=g).to(gpu, torch.bfloat16)
    b = torch.randint(-4, 5, ((N, K) if tb else (K, N)), generator=g).to(gpu, torch.bfloat16)
    y = bf16.gemm(a, b, ta, tb, out_dtype=torch.float32)
    assert torch.equal(y, _ref(a, b, ta, tb))


def test_gemm_identity_asymmetric(gpu):
    I = torch.eye(128, device=gpu, dtype=torch.bfloat16)
    B = (torch.arange(128 * 128, device=gpu) % 251).float().view(128, 128).to(torch.bfloat16)
    assert torch.equal(bf16.gemm(I, B, out_dtype=torch.float32), B.float())
    assert torch.equal(bf16.gemm(B, I, out_dtype=torch.float32), B.float())
    assert torch.equal(bf16.gemm(I, B.t().contiguous(), False, True, out_dtype=torch.float32),
                       B.float())


@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False)])
@pytest.mark.parametrize("M,N,K", [(200, 136, 128), (1000, 768, 768), (64, 3072, 64), (8, 8, 64)])
def test_gemm_random_edges(gpu, ta, tb, M, N, K):
    a = _rand(*((K, M) if ta else (M, K)), dev=gpu, seed=1)
    b = _rand(*((N, K) if tb else (K, N)), dev=gpu, seed=2)
    y = bf16.gemm(a, b, ta, tb, out_dtype=torch.float32)
    ref = _ref(a, b, ta, tb)
    assert (y - ref).abs().max().item() < 1e-5 * K
    yb = bf16.gemm(a, b, ta, tb)
    assert yb.dtype == torch.bfloat16
    assert torch.allclose(yb.float(), ref, rtol=1e-2, atol=1e-2)


def test_gemm_epilogue_bias_gelu_aux_residual(gpu):
    M, N, K = 300, 256, 128
    x = _rand(M, K, dev=gpu, seed=3)
    w = _rand(N, K, dev=gpu, seed=4, scale=0.3)
    bias = torch.randn(N, device=gpu)
    res = _rand(M, N, dev=gpu, seed=5)
    aux = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    y = bf16.gemm(x, w, False, True, bias=bias, act="gelu", aux_out=aux, residual=res,
                  out_dtype=torch.float32)
    u = x.float() @ w.float().t() + bias
    assert torch.allclose(aux.float(), u, rtol=1e-2, atol=1e-2)
    ref = torch.nn.functional.gelu(u, approximate="tanh") + res.float()
    assert (y - ref).abs().max().item() < 1e-3


def test_gemm_act_grad_and_beta(gpu):
    M, N, K = 192, 128, 256
    dy = _rand(M, K, dev=gpu, seed=6)
    w = _rand(K, N, dev=gpu, seed=7, scale=0.2)
    u = _rand(M, N, dev=gpu, seed=8, scale=2.0)
    out = torch.randn(M, N, device=gpu)
    out0 = out.clone()
    bf16.gemm(dy, w, act_grad="gelu", aux_in=u, out=out, beta=1.0)
    ref = (dy.float() @ w.float()) * bf16._gelu_grad_ref(u.float()) + out0
    assert (out - ref).abs().max().item() < 1e-3
    r = bf16.gemm(dy, w, act_grad="relu", aux_in=u, out_dtype=torch.float32)
    assert (r - (dy.float() @ w.float()) * (u.float() > 0)).abs().max().item() < 1e-3


@pytest.mark.parametrize("cfg", [-1, 0, 5])
@pytest.mark.parametrize("M,N,K", [(300, 260, 128), (1024, 1024, 256)])
def test_gemm_gelu_dsave_and_mul(gpu, cfg, M, N, K):
    # act "gelu_dsave": GELU output + gelu'(pre-activation) in aux_out (ragged N = 260 takes the
    # per-element tail path); act_grad "mul": the backward multiplies by that stored derivative
    from distributedtensorflowexample_amd.ops._ext import hip
    x = _rand(M, K, dev=gpu, seed=13)
    w = _rand(N, K, dev=gpu, seed=14, scale=0.3)
    bias = torch.randn(N, device=gpu)
    Np = (N + 7) // 8 * 8  # (row strides must be multiples of 8 elements)
    gp = torch.empty(M, Np, device=gpu, dtype=torch.bfloat16)[:, :N]
    y = torch.empty(M, Np, device=gpu)[:, :N]
    hip().gemm_bf16_set_cfg(cfg)
    try:
        bf16.gemm(x, w, False, True, bias=bias, act="gelu_dsave", aux_out=gp, out=y)
        u = x.float() @ w.float().t() + bias
        assert (y - torch.nn.functional.gelu(u, approximate="tanh")).abs().max().item() < 1e-3
        assert torch.allclose(gp.float(), bf16._gelu_grad_ref(u), rtol=1e-2, atol=1e-2)
        dy = _rand(M, K, dev=gpu, seed=15)
        w2 = _rand(K, N, dev=gpu, seed=16, scale=0.2)
        if N % 8 == 0:
            cs = torch.zeros(N, device=gpu)
            d = bf16.gemm(dy, w2, act_grad="mul", aux_in=gp, out_dtype=torch.float32, colsum=cs)
            ref = (dy.float() @ w2.float()) * gp.float()
            assert (d - ref).abs().max().item() < 1e-3
            assert (cs - ref.sum(0)).abs().max().item() < 1e-3 * M ** 0.5
    finally:
        hip().gemm_bf16_set_cfg(-1)
    with pytest.raises(ValueError):
        bf16.gemm(x, w, False, True, act="gelu_dsave")


@pytest.mark.parametrize("u", [4, 8])  # rows in flight per thread (DTFX_COLSUM_U)
@pytest.mark.parametrize("M,N", [(37, 300), (5000, 300), (2432, 30522)])
def test_colsum_bf16(gpu, M, N, u):
    # (2432 x 30522: the MLM decoder bias gradient; rows split over blocks, atomics)
    from distributedtensorflowexample_amd.ops._ext import hip

    g = _rand(M, N, dev=gpu, seed=9)
    hip().colsum_set_rows_in_flight(u)
    try:
        s = bf16.colsum(g)
        acc = torch.ones(N, device=gpu)
        bf16.colsum(g, out=acc, beta=1.0)
        torch.cuda.synchronize()
    finally:
        hip().colsum_set_rows_in_flight(0)
    assert (s - g.float().sum(0)).abs().max().item() < 1e-3 * (M ** 0.5)
    assert (acc - 1 - g.float().sum(0)).abs().max().item() < 1e-3 * (M ** 0.5)


@pytest.mark.parametrize("splitk,beta", [(0, 0.0), (3, 1.0), (8, 0.0)])
def test_gemm_splitk_wgrad(gpu, splitk, beta):
    # weight-gradient shape: few output tiles, deep K (dW = dY^T . X)
    T, N, K = 4096, 256, 136
    dy = _rand(T, N, dev=gpu, seed=10)
    x = _rand(T, K, dev=gpu, seed=11)
    out = torch.randn(N, K, device=gpu)
    out0 = out.clone()
    bf16.gemm(dy, x, True, False, out=out, beta=beta, splitk=splitk)
    ref = dy.float().t() @ x.float() + beta * out0
    assert (out - ref).abs().max().item() < 1e-4 * T ** 0.5


@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False)])
def test_bmm_strided(gpu, ta, tb):
    nb, M, N, K = 6, 128, 72, 64
    a = _rand(nb, *((K, M) if ta else (M, K)), dev=gpu, seed=12)
    b = _rand(nb, *((N, K) if tb else (K, N)), dev=gpu, seed=13)
    y = bf16.bmm(a, b, ta, tb, out_dtype=torch.float32, alpha=0.5)
    A = a.float().transpose(1, 2) if ta else a.float()
    B = b.float().transpose(1, 2) if tb else b.float()
    assert (y - 0.5 * torch.bmm(A, B)).abs().max().item() < 1e-4


@pytest.fixture(params=[5, 6], ids=["256x256", "256x192"])
def cfg8(gpu, request):
    """Force an 8-phase tile (256x256 or 256x192) for the duration of a test (then auto)."""
    from distributedtensorflowexample_amd.ops import hip

    hip().gemm_bf16_set_cfg(request.param)
    yield request.param
    hip().gemm_bf16_set_cfg(-1)


@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(512, 512, 64), (512, 256, 128), (256, 512, 192),
                                   (296, 520, 320), (1000, 768, 1024), (8, 8, 64),
                                   (512, 384, 128), (264, 200, 64)])
def test_gemm_8phase_exact_integers(cfg8, gpu, ta, tb, M, N, K):
    """8-phase schedule (one, two, three and many K tiles; odd and even tile counts; ragged
    edges): small-integer operands make every partial sum exact, so a mis-staged half
    image, a wrong buffer parity or a read before its DMA landed shows as a mismatch."""
    g = torch.Generator().manual_seed(M + N + K)
    a = torch.randint(-3, 4, ((K, M) if ta else (M, K)), generator=g).to(gpu, torch.bfloat16)
    b = torch.randint(-3, 4, ((N, K) if tb else (K, N)), generator=g).to(gpu, torch.bfloat16)
    for _ in range(3):  # repeated: a race that lands late only sometimes
        y = bf16.gemm(a, b, ta, tb, out_dtype=torch.float32)
        assert torch.equal(y, _ref(a, b, ta, tb))


def test_gemm_8phase_epilogues_and_splitk(cfg8, gpu):
    M, N, K = 600, 512, 256
    x = _rand(M, K, dev=gpu, seed=13)
    w = _rand(N, K, dev=gpu, seed=14, scale=0.3)
    bias = torch.randn(N, device=gpu)
    res = _rand(M, N, dev=gpu, seed=15)
    aux = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    y = bf16.gemm(x, w, False, True, bias=bias, act="gelu", aux_out=aux, residual=res,
                  out_dtype=torch.float32)
    u = x.float() @ w.float().t() + bias
    assert torch.allclose(aux.float(), u, rtol=1e-2, atol=1e-2)
    assert (y - (torch.nn.functional.gelu(u, approximate="tanh") + res.float())).abs().max() < 1e-3
    # fused column sums (bias gradient) over the quadrant-distributed wave layout
    cs = torch.zeros(N, device=gpu)
    yb = bf16.gemm(x, w, False, True, colsum=cs)
    assert (cs - yb.float().sum(0)).abs().max().item() < 2e-2 * M ** 0.5
    # activation gradient (GELU') + f32 accumulation into C (beta = 1)
    pre = _rand(M, N, dev=gpu, seed=18, scale=2.0)
    c0 = torch.randn(M, N, device=gpu)
    c = c0.clone()
    bf16.gemm(x, w, False, True, act_grad="gelu", aux_in=pre, out=c, beta=1.0)
    u2 = pre.float().requires_grad_()
    gg, = torch.autograd.grad(torch.nn.functional.gelu(u2, approximate="tanh").sum(), u2)
    assert (c - (c0 + (x.float() @ w.float().t()) * gg)).abs().max().item() < 1e-3 * K ** 0.5
    # split-K weight gradient on the large tile
    T = 4096
    dy = _rand(T, 512, dev=gpu, seed=16)
    xx = _rand(T, 256, dev=gpu, seed=17)
    out = torch.zeros(512, 256, device=gpu)
    bf16.gemm(dy, xx, True, False, out=out, splitk=4)
    assert (out - dy.float().t() @ xx.float()).abs().max().item() < 1e-4 * T ** 0.5


@pytest.mark.parametrize("tb", [True, False])
def test_gemm_persistent_tile_loop_exact_and_epilogue(gpu, tb):
    """The persistent 8-phase tile loop (one block per CU walks tiles vb, vb + 256, ..; the
    next tile's first K tile staged before this tile's epilogue): exact on integers and
    bit-identical to the one-block-per-tile launch, for 1 / 2 / 3 K tiles (the prologue's
    variants), an uneven last round (456 tiles: blocks with 2 and with 1 tile) and ragged M / N
    edges; the epilogues (bias, GELU with aux, residual, column sums) on every tile."""
    from distributedtensorflowexample_amd.ops._ext import hip

    M, N = 19 * 256 - 100, 24 * 256 - 40  # 456 tiles of 256x256 (R = 200: no tail split)
    g = torch.Generator().manual_seed(21)
    for K in (64, 128, 192):
        a = torch.randint(-3, 4, (M, K), generator=g).to(gpu, torch.bfloat16)
        b = torch.randint(-3, 4, ((N, K) if tb else (K, N)), generator=g).to(gpu, torch.bfloat16)
        old = hip().gemm_bf16_set_pers(1)
        try:
            y = bf16.gemm(a, b, False, tb, out_dtype=torch.float32)
            hip().gemm_bf16_set_pers(0)
            y0 = bf16.gemm(a, b, False, tb, out_dtype=torch.float32)
        finally:
            hip().gemm_bf16_set_pers(old)
        assert torch.equal(y, _ref(a, b, False, tb)), K
        assert torch.equal(y, y0), K
    K = 192
    x = _rand(M, K, dev=gpu, seed=22)
    w = _rand(*((N, K) if tb else (K, N)), dev=gpu, seed=23, scale=0.3)
    bias = torch.randn(N, device=gpu)
    res = _rand(M, N, dev=gpu, seed=24)
    outs = []
    for pers in (1, 0):
        aux = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
        cs = torch.zeros(N, device=gpu)
        old = hip().gemm_bf16_set_pers(pers)
        try:
            yb = bf16.gemm(x, w, False, tb, bias=bias, act="gelu", aux_out=aux, residual=res,
                           colsum=cs)
        finally:
            hip().gemm_bf16_set_pers(old)
        outs.append((yb, aux, cs))
    yb, aux, cs = outs[0]
    u = _ref(x, w, False, tb) + bias
    ref = torch.nn.functional.gelu(u, approximate="tanh") + res.float()
    assert torch.allclose(aux.float(), u, rtol=1e-2, atol=2e-2)
    assert torch.allclose(yb.float(), ref, rtol=1e-2, atol=2e-2)
    assert torch.allclose(cs, yb.float().sum(0), rtol=1e-3, atol=0.5)
    assert torch.equal(yb, outs[1][0]) and torch.equal(aux, outs[1][1])


@pytest.mark.parametrize("tb", [False, True])
def test_gemm_tail_split_exact_and_epilogue(gpu, tb):
    """An 8-phase GEMM with one sparse last round (tiles 17 x 16 = 272: one round + 16 tiles)
    runs its last 256 rows on the 128x128 tile (gemm_tail_rows): exact on integers across the
    seam, and the row-local epilogues (bias, GELU with aux, residual, column sums) land on the
    right rows of both parts."""
    M, N, K = 17 * 256, 16 * 256, 128
    g = torch.Generator().manual_seed(11)
    a = torch.randint(-3, 4, (M, K), generator=g).to(gpu, torch.bfloat16)
    b = torch.randint(-3, 4, ((N, K) if tb else (K, N)), generator=g).to(gpu, torch.bfloat16)
    y = bf16.gemm(a, b, False, tb, out_dtype=torch.float32)
    assert torch.equal(y, _ref(a, b, False, tb))
    x = _rand(M, K, dev=gpu, seed=12)
    w = _rand(*((N, K) if tb else (K, N)), dev=gpu, seed=13, scale=0.3)
    bias = torch.randn(N, device=gpu)
    res = _rand(M, N, dev=gpu, seed=14)
    aux = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    cs = torch.zeros(N, device=gpu)
    yb = bf16.gemm(x, w, False, tb, bias=bias, act="gelu", aux_out=aux, residual=res, colsum=cs)
    u = _ref(x, w, False, tb) + bias
    ref = torch.nn.functional.gelu(u, approximate="tanh") + res.float()
    assert torch.allclose(aux.float(), u, rtol=1e-2, atol=2e-2)
    assert torch.allclose(yb.float(), ref, rtol=1e-2, atol=2e-2)
    assert torch.allclose(cs, yb.float().sum(0), rtol=1e-3, atol=0.5)
