"""BERT MLM step on the GPU kernels vs the same step on the CPU reference paths."""
import math

import pytest
import torch

from distributedtensorflowexample_amd.models.bert import BertConfig, BertMLM, synthetic_mlm_batch

pytestmark = pytest.mark.gpu


def test_bert_tiny_gpu_matches_cpu(gpu):
    cfg = BertConfig.tiny()
    mg, mc = BertMLM(cfg, gpu, seed=2), BertMLM(cfg, "cpu", seed=2)
    mc.params.master.copy_(mg.params.master.cpu())
    mc.params.bf.copy_(mg.params.bf.cpu())
    b = synthetic_mlm_batch(cfg, 4, 128, "cpu", seed=3)
    lg, ag = mg.forward_backward(*(t.to(gpu) for t in b[:4]), n_valid=b[4])
    lc, ac = mc.forward_backward(*b[:4], n_valid=b[4])
    assert abs(lg.item() - lc.item()) < 0.01 * lc.item()
    for name in ["encoder/layer_0/attention/qkv/kernel", "encoder/layer_1/output/dense/kernel",
                 "embeddings/word_embeddings", "embeddings/position_embeddings",
                 "cls/predictions/output_bias", "encoder/layer_1/attention/output/LayerNorm/gamma"]:
        g, r = mg.params.G(name).cpu().flatten(), mc.params.G(name).flatten()
        cos = torch.dot(g, r) / (g.norm() * r.norm() + 1e-30)
        assert cos > 0.99, (name, cos.item())


def test_bert_trainer_graph_replay_matches_eager(gpu):
    from distributedtensorflowexample_amd.train.bert_trainer import BertTrainer

    cfg = BertConfig.tiny()
    a = BertTrainer(cfg, 4, 128, gpu, lr=1e-3)
    b = BertTrainer(cfg, 4, 128, gpu, lr=1e-3)
    a.run(4, use_graph=False)
    b.run(4, use_graph=True)
    # f32 atomics (LayerNorm / embedding / split-K gradients) make the runs differ in the
    # last bits of some gradients; Adam normalises by sqrt(v), so a parameter whose gradient
    # is ~0 can move by up to lr per step either way.  Require bulk agreement + bounded tail.
    # (split-K weight gradients -- one wave of resident blocks -- add 3..14 partial sums per
    # element in arrival order, so a few tenths of a percent of the near-zero-gradient
    # parameters take Adam's +-lr steps differently)
    d = (a.model.params.master - b.model.params.master).abs()
    assert (d <= 2e-5).float().mean() > 0.99
    assert d.max() <= 4 * 1e-3 * 1.01
    assert a.step_count == b.step_count == 4
    la, _ = a.stats()
    lb, _ = b.stats()
    # (absolute: every GEMM of the step is this repo's kernel, whose reduction order does not
    # change under graph capture)
    assert abs(la - lb) < 1e-4


def test_bert_base_step_runs(gpu):
    from distributedtensorflowexample_amd.train.bert_trainer import BertTrainer

    tr = BertTrainer(BertConfig.base(), 8, 128, gpu)
    tr.run(2)
    loss, acc = tr.stats()
    assert 5.0 < loss < 20.0   # ~ln(30522) = 10.3 at init


def test_bert_fits_fixed_batch(gpu):
    from distributedtensorflowexample_amd.train.bert_trainer import BertTrainer

    tr = BertTrainer(BertConfig.tiny(), 8, 128, gpu, lr=2e-3, data_batches=1)
    tr.run(1)
    l0, _ = tr.stats()
    tr.run(30, use_graph=True)
    l1, _ = tr.stats()
    assert l1 < 0.7 * l0, (l0, l1)


def test_bert_dp_adam_waits_for_each_bucket_reduction(gpu):
    """Sync-DP step ordering on the GPU: AdamW of the body buckets runs after THEIR
    all-reduces (comm-stream event) and overlaps the embedding bucket's; AdamW of the
    embeddings after the whole comm stream.  A fake 2-replica communicator makes every
    reduction slow (a GPU spin) and adds 1.0 to each element, so a reduced gradient is
    (g + 1) / 2 > 0 everywhere and the first Adam step moves EVERY parameter down by about
    lr; an AdamW that ran before its bucket's reduction would see g / 2 and move about half
    of them up."""
    from distributedtensorflowexample_amd.train.bert_trainer import BertTrainer

    class SlowPeer:
        world_size, rank = 2, 0

        def allreduce_sum_(self, t):
            torch.cuda._sleep(2_000_000)  # ~1 ms on the comm stream
            return t.add_(1.0)

        def broadcast_(self, t, root=0):
            return t

    lr = 1e-3
    tr = BertTrainer(BertConfig.tiny(), 4, 128, gpu, comm=SlowPeer(), lr=lr, weight_decay=0.0,
                     zero1=False)  # (the all-reduce path; the sharded one: the test below)
    assert tr.comm_stream is not None
    p0 = tr.model.params.master.clone()
    tr.run(1, use_graph=False)
    torch.cuda.synchronize()
    d = tr.model.params.master - p0
    split = tr.model.params.buckets[1][0]
    for part in (d[split:], d[:split]):  # body (overlapped AdamW), embeddings (after the rest)
        assert (part < -0.9 * lr).float().mean().item() > 0.999


def test_gemm_partials_sum_to_reduced_gradient(gpu):
    """``gemm(.., partials=buf)``: a split weight-gradient GEMM leaves its S planes (split
    order) and does not touch ``out``; their sum equals the reduce-pass result."""
    from distributedtensorflowexample_amd.ops import bf16 as B16

    g = torch.Generator().manual_seed(5)
    for M, N, K in ((768, 3072, 16384), (128, 128, 4096), (768, 768, 16384)):
        dy = (torch.randn(K, M, generator=g) * 0.1).to(gpu, torch.bfloat16)
        x = (torch.randn(K, N, generator=g) * 0.1).to(gpu, torch.bfloat16)
        S = B16.splitk_planes(M, N, K)
        assert S > 1, (M, N, K)
        ref = B16.gemm(dy, x, True, False, out=torch.empty(M, N, device=gpu), beta=0.0)
        out = torch.full((M, N), 7.0, device=gpu)
        parts = torch.zeros(S * M * N, device=gpu)
        B16.gemm(dy, x, True, False, out=out, beta=0.0, partials=parts)
        torch.cuda.synchronize()
        assert bool((out == 7.0).all())           # not written
        acc = parts.view(S, M, N)[0].clone()
        for s in range(1, S):
            acc += parts.view(S, M, N)[s]
        exact = dy.float().t() @ x.float()
        tol = 2e-3 * exact.abs().max().item()
        assert (acc - ref).abs().max().item() <= 1e-6 * exact.abs().max().item() + 1e-7
        assert (acc - exact).abs().max().item() <= tol


def test_bert_splitk_fold_matches_reduce_path(gpu, monkeypatch):
    """One-GPU AdamW summing the split-K planes itself (enable_splitk_fold) trains like the
    reduce-pass path: same loss, parameters within the f32-atomics tolerance of the
    eager/graph comparison above."""
    from distributedtensorflowexample_amd.train.bert_trainer import BertTrainer

    cfg = BertConfig.tiny()
    monkeypatch.setenv("DTFX_BERT_FOLD", "0")
    a = BertTrainer(cfg, 32, 128, gpu, lr=1e-3)
    a.init_master = a.model.params.master.clone()
    monkeypatch.setenv("DTFX_BERT_FOLD", "1")
    b = BertTrainer(cfg, 32, 128, gpu, lr=1e-3)
    assert a.model._segs is None and b.model._segs is not None
    assert b.model._segs.shape[0] == 4 * cfg.layers
    a.run(3, use_graph=False)
    b.run(3, use_graph=True)
    d = (a.model.params.master - b.model.params.master).abs()
    assert (d <= 2e-5).float().mean() > 0.99
    # (an elementwise max bound is vacuous here: 3 AdamW steps at lr 1e-3 move a parameter at
    # most ~3e-3, and a near-zero gradient's sign may legitimately differ between the two
    # summation orders) -- the moved parameters as a whole must agree to f32-rounding level
    moved = (a.model.params.master - a.init_master).abs()
    assert d.sum() <= 1e-3 * moved.sum()
    la, _ = a.stats()
    lb, _ = b.stats()
    assert abs(la - lb) < 1e-3 * abs(la)
    # the folded gradients, materialised, match the reduce path's gradients of one step
    a.run(1, use_graph=False)
    b.run(1, use_graph=False)
    b.model.materialize_grads()
    for name in b.model._parts:
        ga, gb = a.model.params.G(name).flatten(), b.model.params.G(name).flatten()
        cos = torch.dot(ga, gb) / (ga.norm() * gb.norm() + 1e-30)
        assert cos > 0.999, (name, cos.item())


def test_bert_splitk_fold_rejects_other_token_count(gpu, monkeypatch):
    """The fold's planes are sized for one token count: a step with another batch x seq (whose
    weight-gradient GEMMs would split differently, or not at all) must raise, not let AdamW
    sum stale planes."""
    from distributedtensorflowexample_amd.models.bert import synthetic_mlm_batch
    from distributedtensorflowexample_amd.ops import bf16 as B16

    cfg = BertConfig.tiny()
    m = BertMLM(cfg, gpu)
    assert m.enable_splitk_fold(32 * 128) > 0
    ids, tt, pos, lab, nv = synthetic_mlm_batch(cfg, 8, 128, gpu)
    with pytest.raises(ValueError, match="split-K fold"):
        m.forward_backward(ids, tt, pos, lab, n_valid=nv)
    # the GEMM-level guard: a partials buffer sized for another plane count
    name = next(iter(m._parts))
    W = m.params.G(name)
    M, N = W.shape
    dy = torch.randn(8 * 128, M, device=gpu).to(torch.bfloat16)
    x = torch.randn(8 * 128, N, device=gpu).to(torch.bfloat16)
    with pytest.raises(ValueError, match="partial"):
        B16.gemm(dy, x, True, False, out=W, beta=0.0, partials=m._parts[name])


def test_bert_overlapped_adam_matches_one_launch(gpu, monkeypatch):
    """One GPU: each bucket's AdamW on a third stream as soon as the bucket is final (overlapping
    the rest of the backward) gives the one-launch-after-backward result."""
    from distributedtensorflowexample_amd.train.bert_trainer import BertTrainer

    cfg = BertConfig.tiny()
    monkeypatch.delenv("DTFX_BERT_OPT_OVERLAP", raising=False)
    a = BertTrainer(cfg, 32, 128, gpu, lr=1e-3)  # default: AdamW after the backward
    a.init_master = a.model.params.master.clone()
    monkeypatch.setenv("DTFX_BERT_OPT_OVERLAP", "1")
    b = BertTrainer(cfg, 32, 128, gpu, lr=1e-3)
    assert a.opt_stream is None and b.opt_stream is not None
    a.run(3, use_graph=False)
    b.run(3, use_graph=True)
    d = (a.model.params.master - b.model.params.master).abs()
    assert (d <= 2e-5).float().mean() > 0.99
    # (an elementwise max bound is vacuous here: 3 AdamW steps at lr 1e-3 move a parameter at
    # most ~3e-3, and a near-zero gradient's sign may legitimately differ between the two
    # summation orders) -- the moved parameters as a whole must agree to f32-rounding level
    moved = (a.model.params.master - a.init_master).abs()
    assert d.sum() <= 1e-3 * moved.sum()
    assert int(a.step_t.item()) == int(b.step_t.item()) == 4
    la, _ = a.stats()
    lb, _ = b.stats()
    assert abs(la - lb) < 1e-3 * abs(la)


def test_bert_zero1_step_captures_and_runs(gpu):
    """The owner-sharded AdamW path (world > 1 default) under hipGraph capture: the comm-stream
    gathers at the step's start, per-bucket reduce-scatter events, the shard AdamW -- rank 0 of
    a simulated world-2 job (parallel.xgmi.SimulatedPeersComm: the real bw kernel halves over
    local peers; the values are a timing harness's, so only the shape and finiteness are
    checked here; the numerics are tests/test_dp_models_gloo.py's)."""
    from distributedtensorflowexample_amd.parallel.xgmi import SimulatedPeersComm
    from distributedtensorflowexample_amd.train.bert_trainer import BertTrainer

    comm = SimulatedPeersComm(2, 1 << 20, device=gpu)
    tr = BertTrainer(BertConfig.tiny(), 4, 128, gpu, comm=comm, lr=1e-3)
    assert tr.zero1 and tr.model.params.numel % (64 * 2) == 0
    tr.run(3, use_graph=True)
    torch.cuda.synchronize()
    comm.check()
    loss, _ = tr.stats()
    assert math.isfinite(loss)
    tr.sync_params()
    assert bool(torch.isfinite(tr.model.params.master).all())


def test_zero_grad_one_launch_matches_views(gpu, monkeypatch):
    """The per-step zeroing of the accumulated gradient slots as ONE zero_ranges launch (the
    default) zeroes exactly the ranges the strided per-view fills do, and nothing else."""
    from distributedtensorflowexample_amd.models.bert import FlatParams

    cfg = BertConfig.tiny()
    outs = []
    for env in ("1", "0"):
        monkeypatch.setenv("DTFX_ZERO_RANGES", env)
        p = FlatParams(cfg, gpu, seed=1)
        p.grad.copy_(torch.arange(p.grad.numel(), device=gpu, dtype=torch.float32) + 1)
        p.zero_grad()
        assert (p._zero_tab is not None) == (env == "1")
        outs.append(p.grad.clone())
    assert torch.equal(outs[0], outs[1])
    assert (outs[0] == 0).any() and (outs[0] != 0).any()
