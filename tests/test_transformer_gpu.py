"""Transformer HIP kernels vs the f32 PyTorch reference of the same op (1 GPU)."""

import pytest
import torch

from distributedtensorflowexample_amd.ops import _ext
from distributedtensorflowexample_amd.ops import transformer as T

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def _r(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale)


# backward variants: row slots per wave of the generic kernel (DTFX_LN_SLOTS 2 / 3) and the
# H = 768 kernel (DTFX_LN_H768=1; the generic one at every other H)
@pytest.mark.parametrize("slots", [2, 3, "h768"])
@pytest.mark.parametrize("Tn,H", [(300, 768), (37, 136), (70, 2048), (129, 1000), (16384, 768)])
def test_layernorm_fwd_bwd(gpu, Tn, H, slots):
    # (row counts off the 16-row blocks of the 4-rows-per-wave forward; 1..4 column chunks;
    # 16384 x 768: the BERT shape, 64 rows per block)
    x = _r(Tn, H, seed=1).to(BF)
    gamma, beta = _r(H, seed=2) * 0.1 + 1, _r(H, seed=3) * 0.1
    y, mean, rstd = T.layernorm_fwd(x.to(gpu), gamma.to(gpu), beta.to(gpu))
    yr, mr, rr = T.layernorm_fwd(x, gamma, beta)
    assert torch.allclose(mean.cpu(), mr, atol=1e-5) and torch.allclose(rstd.cpu(), rr, rtol=1e-4)
    assert (y.cpu().float() - yr.float()).abs().max() < 3e-2
    dy, dres = _r(Tn, H, seed=4).to(BF), _r(Tn, H, seed=5).to(BF)
    dg, db = torch.zeros(H, device=gpu), torch.zeros(H, device=gpu)
    hip = _ext.hip()
    hip.ln_bwd_set_slots(2 if slots == "h768" else slots)
    hip.ln_bwd_set_h768(1 if slots == "h768" else 0)
    try:
        dx = T.layernorm_bwd(dy.to(gpu), x.to(gpu), mean, rstd, gamma.to(gpu), dg, db,
                             dres.to(gpu))
        torch.cuda.synchronize()
    finally:
        hip.ln_bwd_set_slots(-1)
        hip.ln_bwd_set_h768(-1)
    dgr, dbr = torch.zeros(H), torch.zeros(H)
    dxr = T.layernorm_bwd(dy, x, mr, rr, gamma, dgr, dbr, dres)
    assert (dx.cpu().float() - dxr.float()).abs().max() < 5e-2
    assert torch.allclose(dg.cpu(), dgr, atol=1e-2, rtol=1e-3)
    assert torch.allclose(db.cpu(), dbr, atol=1e-2, rtol=1e-3)


@pytest.mark.parametrize("B", [3, 70])  # 70: the position / type gradient split over the batch
def test_embedding_fwd_bwd(gpu, B):
    S, H, V = 40, 256, 1000
    ids = torch.randint(0, V, (B * S,), dtype=torch.int32)
    tt = torch.randint(0, 2, (B * S,), dtype=torch.int32)
    word, pos, typ = _r(V, H, seed=6).to(BF), _r(64, H, seed=7).to(BF), _r(2, H, seed=8).to(BF)
    gamma, beta = torch.ones(H), torch.zeros(H)
    out = T.embed_ln_fwd(ids.to(gpu), tt.to(gpu), word.to(gpu), pos.to(gpu), typ.to(gpu),
                         gamma.to(gpu), beta.to(gpu), S)
    ref = T.embed_ln_fwd(ids, tt, word, pos, typ, gamma, beta, S)
    assert torch.equal(out[0].cpu(), ref[0])
    assert (out[1].cpu().float() - ref[1].float()).abs().max() < 3e-2
    dx = _r(B * S, H, seed=9).to(BF)
    g = [torch.zeros(V, H), torch.zeros(64, H), torch.zeros(2, H)]
    gg = [t.to(gpu) for t in g]
    T.embed_bwd(ids.to(gpu), tt.to(gpu), dx.to(gpu), *gg, B, S)
    T.embed_bwd(ids, tt, dx, *g, B, S)
    for a, b in zip(gg, g):
        assert torch.allclose(a.cpu(), b, atol=1e-3)


# 3 / 4: persistent (4: 3 blocks, 4 pairs each); 5: the two-halves kernel and the P-through-LDS
# forward with the XOR-swizzled LDS images (opt-in DTFX_ATTN_SWZ=1); 6: the two-halves kernel
# and the P-through-LDS forward (DTFX_ATTN_FWD=0); 7: the two-halves kernel with the opt-in V-row
# L2 warm-up (DTFX_ATTN_BWD_PF=1).  Variants 0-4 and 7 run the default forward with P in
# registers (attn_fwd_rp_kernel).
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 6, 7])
@pytest.mark.parametrize("S,masked", [(128, False), (128, True), (77, True), (64, False), (33, True)])
def test_attention_fwd_bwd(gpu, S, masked, variant):
    B, nh = 3, 4
    qkv = _r(B * S, 3 * nh * 64, seed=10).to(BF)
    kmask = None
    if masked:
        valid = torch.tensor([S, S - 5, S // 2])
        kmask = torch.where(torch.arange(S)[None, :] < valid[:, None], 0.0, -10000.0)
    hip = _ext.hip()
    hip.attn_set_swizzle(1 if variant == 5 else 0)
    hip.attn_fwd_set_variant(0 if variant in (5, 6) else 1)
    hip.attn_bwd_set_pf(1 if variant == 7 else 0)
    try:
        o, lse = T.attn_fwd(qkv.to(gpu), B, S, nh, kmask.to(gpu) if masked else None)
        orf, lser = T.attn_fwd(qkv, B, S, nh, kmask)
        assert (o.cpu().float() - orf.float()).abs().max() < 2e-2
        assert (lse.cpu().view(B, nh, -1)[..., :S] - lser.view(B, nh, -1)[..., :S]).abs().max() < 1e-3
        dout = _r(B * S, nh * 64, seed=11).to(BF)
        hip.attn_bwd_set_variant(2 if variant >= 5 else variant)
        dq = T.attn_bwd(qkv.to(gpu), o, dout.to(gpu), lse, B, S, nh, kmask.to(gpu) if masked else None)
        torch.cuda.synchronize()
    finally:
        hip.attn_bwd_set_variant(-1)
        hip.attn_bwd_set_pf(-1)
        hip.attn_set_swizzle(-1)
        hip.attn_fwd_set_variant(-1)
    dqr = T.attn_bwd(qkv, o.cpu(), dout, lse.cpu(), B, S, nh, kmask)
    err = (dq.cpu().float() - dqr.float()).abs().max().item()
    assert err < 3e-2 * max(1.0, dqr.float().abs().max().item()), err


def test_adam_mixed_and_cast(gpu):
    n = 4096
    p, g = _r(n, seed=12), _r(n, seed=13)
    m, v = torch.zeros(n), torch.zeros(n)
    P, G, M, Vv = (t.to(gpu) for t in (p, g, m, v))
    pb = torch.empty(n, device=gpu, dtype=BF)
    for step in (1, 2, 3):
        T.adam_mixed(P, G, M, Vv, pb, 1e-3, step, gscale=0.5)
        T.adam_mixed(p, g, m, v, None, 1e-3, step, gscale=0.5)
    assert torch.allclose(P.cpu(), p, atol=1e-6, rtol=1e-5)
    assert torch.equal(pb.cpu(), P.cpu().to(BF))
    assert torch.equal(T.cast_bf16(G).cpu(), g.to(BF))


# regs: the bf16 kernel holding the row in registers (default) or the two-pass one; the
# 30522 / 30528 case is the BERT vocabulary (15 chunks of 8 per thread, a 2-element tail)
@pytest.mark.parametrize("regs", [1, 0])
@pytest.mark.parametrize("dtype,N,C,ld", [(torch.float32, 70, 1003, 1024), (BF, 70, 1003, 1024),
                                          (BF, 37, 30522, 30528), (BF, 5, 7, 8)])
def test_mlm_xent_matches_reference(gpu, dtype, N, C, ld, regs):
    # bf16 logits: the kernel reads them as stored, the reference gets the same rounded values
    logits = (_r(N, ld, seed=20) * 3).to(dtype)
    lab = torch.randint(0, C, (N,), dtype=torch.int32)
    lab[min(5, N - 1)] = -100
    lab[0] = int(logits[0, :C].float().argmax())  # at least one correct prediction
    hip = _ext.hip()
    hip.xent_set_regs(regs)
    try:
        lg, cg, dg = T.mlm_xent(logits.to(gpu), lab.to(gpu), C, 1 / 69)
        torch.cuda.synchronize()
    finally:
        hip.xent_set_regs(-1)
    lr, cr, dr = T.mlm_xent(logits, lab, C, 1 / 69)
    assert torch.allclose(lg.cpu(), lr, atol=1e-4)
    assert torch.equal(cg.cpu(), cr)
    assert (dg.cpu().float() - dr.float()).abs().max() < 1e-4
    assert (dg[:, C:] == 0).all()


def test_fused_bias_grads(gpu):
    from distributedtensorflowexample_amd.ops import bf16

    Tn, H = 256, 128
    x = _r(Tn, H, seed=21).to(BF)
    gamma = torch.ones(H)
    y, mean, rstd = T.layernorm_fwd(x, gamma, torch.zeros(H))
    dy = _r(Tn, H, seed=22).to(BF)
    s = torch.zeros(H, device=gpu)
    dx = T.layernorm_bwd(dy.to(gpu), x.to(gpu), mean.to(gpu), rstd.to(gpu), gamma.to(gpu),
                         torch.zeros(H, device=gpu), torch.zeros(H, device=gpu), dxsum=s)
    # f32 sums vs sums of the bf16-rounded outputs: ~sqrt(T) * 2^-9 apart
    assert torch.allclose(s.cpu(), dx.cpu().float().sum(0), atol=0.15)
    w = _r(64, H, seed=23).to(BF).to(gpu)
    cs = torch.zeros(64, device=gpu)
    out = bf16.gemm(dx, w, False, True, colsum=cs, out_dtype=torch.float32)
    assert torch.allclose(cs, out.sum(0), atol=1e-3, rtol=1e-4)
    B, S, nh = 2, 128, 2
    qkv = _r(B * S, 3 * nh * 64, seed=24).to(BF).to(gpu)
    o, lse = T.attn_fwd(qkv, B, S, nh)
    db = torch.zeros(3 * nh * 64, device=gpu)
    dq = T.attn_bwd(qkv, o, _r(B * S, nh * 64, seed=25).to(BF).to(gpu), lse, B, S, nh, dbias=db)
    assert torch.allclose(db, dq.float().sum(0), atol=0.15, rtol=1e-2)


@pytest.mark.parametrize("S,masked,force", [(512, True, False), (200, False, False),
                                            (77, True, True), (128, False, True)])
def test_flash_attention_fwd_bwd(gpu, monkeypatch, S, masked, force):
    if force:
        monkeypatch.setenv("DTFX_ATTN", "flash")
    B, nh = 2, 3
    qkv = _r(B * S, 3 * nh * 64, seed=30).to(BF)
    kmask = None
    if masked:
        valid = torch.tensor([S, S - 37])
        kmask = torch.where(torch.arange(S)[None, :] < valid[:, None], 0.0, -10000.0)
    o, lse = T.attn_fwd(qkv.to(gpu), B, S, nh, kmask.to(gpu) if masked else None)
    orf, lser = T.attn_fwd(qkv, B, S, nh, kmask)
    assert (o.cpu().float() - orf.float()).abs().max() < 2e-2
    assert (lse.cpu().view(B, nh, -1)[..., :S] - lser.view(B, nh, -1)[..., :S]).abs().max() < 1e-3
    dout = _r(B * S, nh * 64, seed=31).to(BF)
    db = torch.zeros(3 * nh * 64, device=gpu)
    dq = T.attn_bwd(qkv.to(gpu), o, dout.to(gpu), lse, B, S, nh, kmask.to(gpu) if masked else None,
                    dbias=db)
    dbr = torch.zeros(3 * nh * 64)
    dqr = T.attn_bwd(qkv, o.cpu(), dout, lse.cpu(), B, S, nh, kmask, dbias=dbr)
    err = (dq.cpu().float() - dqr.float()).abs().max().item()
    assert err < 3e-2 * max(1.0, dqr.float().abs().max().item()), err
    assert torch.allclose(db.cpu(), dbr, atol=0.2, rtol=2e-2)


@pytest.mark.parametrize("S", [128, 77])
def test_attention_fwd_register_p_matches_lds_p(gpu, S):
    """The forward with P in registers (attn_fwd_rp_kernel: scores formed transposed, P . V's A
    operand straight from the accumulators) against the P-through-LDS kernel on the same
    inputs: outputs within two bf16 roundings (the scores' MFMA operands are swapped and P . V
    sums its keys in another order, so a P element can round the other way), log-sum-exp
    within f32 rounding."""
    B, nh = 8, 12
    qkv = (_r(B * S, 3 * nh * 64, seed=20) * 2).to(BF).to(gpu)
    valid = torch.randint(S // 2, S + 1, (B,), generator=torch.Generator().manual_seed(3))
    kmask = torch.where(torch.arange(S)[None, :] < valid[:, None], 0.0, -10000.0).to(gpu)
    hip = _ext.hip()
    res = []
    try:
        for v in (1, 0):
            hip.attn_fwd_set_variant(v)
            res.append(T.attn_fwd(qkv, B, S, nh, kmask))
    finally:
        hip.attn_fwd_set_variant(-1)
    (o1, l1), (o0, l0) = res
    d = (o1.float() - o0.float()).abs()
    assert (d <= 2 ** -6 * o0.float().abs() + 4e-3).all(), d.max().item()
    l1v, l0v = l1.view(B, nh, -1)[..., :S], l0.view(B, nh, -1)[..., :S]
    assert (l1v - l0v).abs().max().item() < 1e-4
