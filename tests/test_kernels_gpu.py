"""Numerics of every HIP kernel against a float64 PyTorch reference (1 GPU)."""
import pytest
import torch

from distributedtensorflowexample_amd.ops import init, mlp_step, nn, optim

pytestmark = pytest.mark.gpu


def _rand(*shape, dev, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return ((torch.rand(*shape, generator=g) * 2 - 1) * scale).to(dev)


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(100, 100, 784), (37, 129, 65), (64, 64, 16), (1, 10, 3)])
def test_gemm_matches_fp64(gpu, ta, tb, M, N, K):
    a = _rand(*((K, M) if ta else (M, K)), dev=gpu, seed=1)
    b = _rand(*((N, K) if tb else (K, N)), dev=gpu, seed=2)
    y = nn.gemm(a, b, trans_a=ta, trans_b=tb)
    A = a.double().t() if ta else a.double()
    B = b.double().t() if tb else b.double()
    ref = A @ B
    tol = 2e-6 * (A.abs() @ B.abs()).max().item() + 1e-6
    assert (y.double() - ref).abs().max().item() < tol


def test_gemm_identity_asymmetric(gpu):
    # A = I with an ASYMMETRIC B catches a transposed C/D write (guide §3).
    I = torch.eye(48, device=gpu)
    B = torch.arange(48 * 48, device=gpu, dtype=torch.float32).view(48, 48)
    assert torch.equal(nn.gemm(I, B), B)
    assert torch.equal(nn.gemm(B, I), B)


@pytest.mark.parametrize("act", ["sigmoid", "relu", "gelu", None])
def test_gemm_epilogues(gpu, act):
    x = _rand(70, 90, dev=gpu, seed=3)
    w = _rand(33, 90, dev=gpu, seed=4, scale=0.3)
    b = _rand(33, dev=gpu, seed=5)
    y = nn.gemm(x, w, trans_b=True, bias=b, act=act)
    z = x.double() @ w.double().t() + b.double()
    ref = nn._act_ref(z, nn._act_id(act))
    assert (y.double() - ref).abs().max().item() < 2e-5
    # backward epilogue + beta accumulation
    dy = _rand(70, 33, dev=gpu, seed=6)
    aux = z.float() if act == "gelu" else y
    out = _rand(70, 90, dev=gpu, seed=7)
    out0 = out.clone()
    eye = torch.eye(33, device=gpu)
    dz = nn.gemm(dy, eye, act=act, aux=aux, act_grad=True)
    refdz = nn._act_grad_ref(dy.double(), aux.double(), nn._act_id(act))
    assert (dz.double() - refdz).abs().max().item() < 1e-5
    g = nn.gemm(dy, w, beta=0.5, out=out)
    refg = dy.double() @ w.double() + 0.5 * out0.double()
    assert (g.double() - refg).abs().max().item() < 2e-5


def test_dense_autograd(gpu):
    x = _rand(50, 40, dev=gpu, seed=8).requires_grad_()
    w = _rand(20, 40, dev=gpu, seed=9).requires_grad_()
    b = _rand(20, dev=gpu, seed=10).requires_grad_()
    y = nn.dense(x, w, b, "sigmoid")
    (y * torch.arange(20, device=gpu)).sum().backward()
    x64, w64, b64 = (t.detach().double().cpu().requires_grad_() for t in (x, w, b))
    y64 = torch.sigmoid(x64 @ w64.t() + b64)
    (y64 * torch.arange(20).double()).sum().backward()
    for t, r in ((x, x64), (w, w64), (b, b64)):
        assert (t.grad.double().cpu() - r.grad).abs().max().item() < 1e-4


@pytest.mark.parametrize("dense_labels", [False, True])
def test_softmax_xent(gpu, dense_labels):
    N, C = 300, 10
    logits = _rand(N, C, dev=gpu, seed=11, scale=5)
    lab = torch.randint(0, C, (N,), generator=torch.Generator().manual_seed(0)).to(gpu)
    labels = torch.nn.functional.one_hot(lab, C).float() if dense_labels else lab.int()
    loss, d, correct = nn.softmax_xent_stats(logits, labels)
    l64 = logits.double().cpu()
    ref_loss = torch.nn.functional.cross_entropy(l64, lab.cpu(), reduction="none")
    assert (loss.double().cpu() - ref_loss).abs().max().item() < 1e-5
    ref_d = (torch.softmax(l64, 1) - torch.nn.functional.one_hot(lab.cpu(), C).double()) / N
    assert (d.double().cpu() - ref_d).abs().max().item() < 1e-7
    assert torch.equal(correct.cpu(), (l64.argmax(1) == lab.cpu()).float())


def test_optimizers(gpu):
    n = 1027  # float4 body + scalar tail
    p = _rand(n, dev=gpu, seed=12)
    g = _rand(n, dev=gpu, seed=13)
    pc, gc = p.cpu().clone(), g.cpu().clone()
    optim.sgd_(p, g, 0.1, weight_decay=0.01)
    optim.sgd_(pc, gc, 0.1, weight_decay=0.01)
    assert (p.cpu() - pc).abs().max().item() < 1e-6
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    mc, vc = m.cpu().clone(), v.cpu().clone()
    for s in (1, 2, 3):
        optim.adam_(p, g, m, v, 1e-3, s, weight_decay=0.01)
        optim.adam_(pc, gc, mc, vc, 1e-3, s, weight_decay=0.01)
    assert (p.cpu() - pc).abs().max().item() < 1e-5
    buf, bufc = torch.zeros_like(p), torch.zeros(n)
    optim.momentum_(p, g, buf, 0.1, 0.9, nesterov=True)
    optim.momentum_(pc, gc, bufc, 0.1, 0.9, nesterov=True)
    assert (p.cpu() - pc).abs().max().item() < 1e-5


def test_philox_init(gpu):
    t = torch.empty(1 << 20, device=gpu)
    init.fill_(t, "normal", 0.0, 1.0, seed=7)
    assert abs(t.mean().item()) < 5e-3 and abs(t.std().item() - 1) < 5e-3
    t2 = torch.empty_like(t)
    init.fill_(t2, "normal", 0.0, 1.0, seed=7)
    assert torch.equal(t, t2)  # counter-based => reproducible on every rank
    init.fill_(t, "truncated_normal", 0.0, 0.02, seed=3)
    assert t.abs().max().item() <= 0.04 + 1e-7
    init.fill_(t, "uniform", -1.0, 2.0, seed=3)
    assert t.min().item() >= -1.0 and t.max().item() < 2.0


def _mlp_setup(gpu, B, nb, seed=0):
    p = torch.empty(mlp_step.NPARAM, device=gpu)
    init.fill_(p, "normal", 0.0, 1.0, seed=seed)
    p[mlp_step.OFF_B1:mlp_step.OFF_W2].zero_()
    p[mlp_step.OFF_B2:].zero_()
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(nb * B, 784, generator=g).to(gpu)
    y = torch.randint(0, 10, (nb * B,), generator=g).to(gpu).int()
    return p, x, y


@pytest.mark.parametrize("B", [100, 1, 37, 256])
def test_mlp_fused_step_grads(gpu, B):
    p, x, y = _mlp_setup(gpu, B, 1)
    ws = mlp_step.StepWorkspace(B, gpu)
    grad = torch.zeros_like(p)
    mlp_step.step_grad(p, x, y, ws, grad)
    torch.cuda.synchronize()
    g64, loss, acc = mlp_step.reference_step(p.double().cpu(), x.double().cpu(), y.cpu())
    err = (grad.double().cpu() - g64).abs().max().item()
    assert err < 1e-4 * max(1.0, g64.abs().max().item()), err
    st = ws.stats[0].cpu()
    assert abs(st[0].item() - loss.item()) < 1e-3 * max(1.0, loss.item())
    assert abs(st[1].item() - acc.item()) < 1e-6
    assert ws.global_step() == 1


def test_mlp_fused_small_weights(gpu):
    """Non-saturated regime (small weights): sigmoid' and dW2/db2 paths all live."""
    B = 100
    p, x, y = _mlp_setup(gpu, B, 1)
    p.mul_(0.05)
    ws = mlp_step.StepWorkspace(B, gpu)
    grad = torch.zeros_like(p)
    mlp_step.step_grad(p, x, y, ws, grad)
    torch.cuda.synchronize()
    g64, _, _ = mlp_step.reference_step(p.double().cpu(), x.double().cpu(), y.cpu())
    for a_, b_ in zip(mlp_step.unflatten(grad.double().cpu()), mlp_step.unflatten(g64)):
        assert (a_ - b_).abs().max().item() < 1e-5 * max(1.0, b_.abs().max().item())


def test_mlp_direct_step_matches_reference(gpu):
    """Single-GPU mode: SGD apply fused into mlp_wgrad, several steps."""
    B, nb, lr, steps = 100, 3, 0.5, 6
    p, x, y = _mlp_setup(gpu, B, nb, seed=2)
    p.mul_(0.1)
    ws = mlp_step.StepWorkspace(B, gpu)
    ref = p.double().cpu()
    xr, yr = x.double().cpu(), y.cpu()
    for s in range(steps):
        sl = slice((s % nb) * B, (s % nb + 1) * B)
        mlp_step.step_direct(p, x[sl], y[sl], ws, lr)
        g, _, _ = mlp_step.reference_step(ref, xr[sl], yr[sl])
        ref = ref - lr * g
    torch.cuda.synchronize()
    assert (p.double().cpu() - ref).abs().max().item() < 1e-4
    assert ws.global_step() == steps


def test_mlp_deferred_apply_multi_step(gpu):
    """Sync-DP mode: gradient written, applied at the start of the next step."""
    B, nb, lr, steps = 100, 3, 0.5, 5
    p, x, y = _mlp_setup(gpu, B, nb, seed=1)
    p.mul_(0.1)
    ws = mlp_step.StepWorkspace(B, gpu)
    cur, spare = p.clone(), torch.empty_like(p)
    grad = torch.zeros_like(p)
    ref = p.double().cpu()
    xr, yr = x.double().cpu(), y.cpu()
    gref = None
    for s in range(steps):
        sl = slice((s % nb) * B, (s % nb + 1) * B)
        if s == 0:
            mlp_step.step_grad(cur, x[sl], y[sl], ws, grad)
        else:
            mlp_step.step_grad(cur, x[sl], y[sl], ws, grad, prev_grad=grad, lr=lr, p_new=spare)
            cur, spare = spare, cur
            ref = ref - lr * gref
        gref, _, _ = mlp_step.reference_step(ref, xr[sl], yr[sl])
        torch.cuda.synchronize()
        assert (cur.double().cpu() - ref).abs().max().item() < 1e-4
        assert (grad.double().cpu() - gref).abs().max().item() < 1e-4
    assert ws.global_step() == steps


@pytest.mark.parametrize("dp", [False, True])
def test_trainer_graph_replay_matches_eager(gpu, dp):
    from distributedtensorflowexample_amd.train.fused_mlp import FusedMLPTrainer

    B, nb = 100, 5
    p, x, y = _mlp_setup(gpu, B, nb, seed=3)
    p.mul_(0.1)
    ar = (lambda g: None) if dp else None
    t1 = FusedMLPTrainer(p, x, y, B, 0.3, allreduce=ar)
    t2 = FusedMLPTrainer(p, x, y, B, 0.3, allreduce=ar)
    t1.max_graph_steps = 4
    t1.run(23, use_graph=True)
    t2.run(23, use_graph=False)
    t1.flush()
    t2.flush()
    torch.cuda.synchronize()
    assert t1.global_step() == t2.global_step() == 23
    assert torch.equal(t1.params, t2.params)
    assert t1.stats() == t2.stats()


@pytest.mark.parametrize("B", [100, 64, 200])
def test_pipelined_trainer_matches_reference_and_three_launch(gpu, B):
    """Two-launch pipelined step (apply of step t-1 fused with the forward of step t):
    same SGD trajectory as the float64 reference and as the three-launch trainer, through
    graph replays, a mid-run flush and the generic-batch kernel variants."""
    from distributedtensorflowexample_amd.train.fused_mlp import FusedMLPTrainer

    nb, lr = 4, 0.3
    p, x, y = _mlp_setup(gpu, B, nb, seed=4)
    p.mul_(0.1)
    tp = FusedMLPTrainer(p, x, y, B, lr)                   # pipelined (default)
    t3 = FusedMLPTrainer(p, x, y, B, lr, pipeline=False)   # three launches
    assert tp.pipelined and not t3.pipelined
    tp.max_graph_steps = 3
    t3.max_graph_steps = 3
    tp.run(6, use_graph=False)
    t3.run(6, use_graph=False)
    # float64 reference of the first 6 steps
    ref = p.double().cpu()
    xr, yr = x.double().cpu(), y.cpu()
    for s in range(6):
        sl = slice((s % nb) * B, (s % nb + 1) * B)
        g, _, _ = mlp_step.reference_step(ref, xr[sl], yr[sl])
        ref = ref - lr * g
    assert tp.global_step() == 6
    tp.flush()
    torch.cuda.synchronize()
    assert (tp.params.double().cpu() - ref).abs().max().item() < 1e-4
    tp.run(11, use_graph=True)  # graph replays after a flush (first step re-primes)
    t3.run(11, use_graph=True)
    tp.flush()
    torch.cuda.synchronize()
    assert tp.global_step() == t3.global_step() == 17
    assert (tp.params - t3.params).abs().max().item() < 1e-5
    lp, ap = tp.stats()
    l3, a3 = t3.stats()
    assert abs(lp - l3) < 1e-4 and ap == a3
    assert torch.allclose(tp.stats_range(0, 17), t3.stats_range(0, 17), atol=1e-4)


def test_host_loop_matches_graph_replay(gpu):
    """FusedMLPTrainer.run_launched (one C++ call issuing every step's kernels) and the
    graph path (with and without host-launched lead steps) walk the dataset identically:
    bit-identical parameters, global_step and stats, across an epoch boundary."""
    from distributedtensorflowexample_amd.data.synthetic import mnist_like_device
    from distributedtensorflowexample_amd.models.mlp import init_params
    from distributedtensorflowexample_amd.train.fused_mlp import FusedMLPTrainer

    p = init_params(gpu, seed=3)
    x, y = mnist_like_device(1300, seed=4, device=gpu)  # 13 batches: runs wrap the epoch
    runs = {}
    for mode in ("graph", "host", "host_flush", "lead"):
        tr = FusedMLPTrainer(p, x, y, 100, 0.05)
        if mode == "graph":
            tr.run(3)
            tr.run(20)
        elif mode == "host":
            tr.run_launched(3)
            tr.run_launched(20)
        elif mode == "host_flush":  # the flush launched by the same call (bench.py's timed region)
            tr.run_launched(3)
            tr.run_launched(20, flush=True)
            assert not tr.pending
        else:
            tr.run(3)
            tr.prepare(20, lead=4)
            tr.run(20, lead=4)
        st = tr.stats_range(0, 23).clone()
        runs[mode] = (tr.flush().clone(), tr.global_step(), st, tr.pos)
    for mode in ("host", "host_flush", "lead"):
        assert torch.equal(runs[mode][0], runs["graph"][0]), mode
        assert runs[mode][1] == runs["graph"][1] == 23
        assert torch.equal(runs[mode][2], runs["graph"][2]), mode
        assert runs[mode][3] == runs["graph"][3] == 23 % 13


@pytest.mark.parametrize("B", [100, 7, 128])
def test_terminal_head_flush_matches_separate_flush_and_fp64(gpu, B):
    """run_launched(K, flush=True) ends on ONE launch that runs the last step's head and the
    apply of its update (mlp_head_flush_kernel).  Against the same steps
    with the flush as its own launch (FusedMLPTrainer.flush): bit-identical parameters,
    global_step and loss / accuracy records, over back-to-back flushed regions of K = 1, 5, 20
    (the hand-off words must reset between launches); and the applied trajectory against an
    fp64 CPU reference of the reference's SGD (worker.py:59-79)."""
    import __graft_entry__ as ge
    from distributedtensorflowexample_amd.data.synthetic import mnist_like_device
    from distributedtensorflowexample_amd.models.mlp import init_params
    from distributedtensorflowexample_amd.train.fused_mlp import FusedMLPTrainer

    from distributedtensorflowexample_amd.ops._ext import hip

    p = init_params(gpu, seed=5)
    nb = 30
    x, y = mnist_like_device(nb * B, seed=6, device=gpu)
    fused = FusedMLPTrainer(p, x, y, B, 0.001)
    sep = FusedMLPTrainer(p, x, y, B, 0.001)
    for k in (1, 5, 20):
        old = hip().mlp_set_flush_fused(1)  # (opt-in: DTFX_MLP_FLUSH_FUSED=1)
        try:
            fused.run_launched(k, flush=True)
        finally:
            hip().mlp_set_flush_fused(old)
        sep.run_launched(k)
        sep.flush()
        assert not fused.pending
        assert torch.equal(fused.params, sep.params), k
    fused.check()  # no hand-off timed out
    sync = fused.ws.buf[-4:].view(torch.int32)
    assert sync.tolist() == [0, 0, 0, 0]  # reset by the last apply block of every launch
    assert fused.global_step() == sep.global_step() == 26
    assert torch.equal(fused.stats_range(0, 26), sep.stats_range(0, 26))
    p_ref, hist_ref = ge.reference_sgd(p, x, y, 0.001, 26, batch=B)
    hist = [tuple(float(v) for v in r) for r in fused.stats_range(0, 26).cpu()]
    ge.check_step_result(p, fused.params, hist, p_ref, hist_ref)


@pytest.mark.parametrize("B", [100, 64, 128, 7])
def test_persistent_trainer_matches_pipelined(gpu, B):
    """The persistent single-launch engine (workgroups hand z1 partials, backprop factors and
    small parameters to each other as epoch-tagged granules) runs the same SGD trajectory as
    the two-launch pipelined step -- parameters within f32 rounding (the compiler may contract
    a different product of a dot into an FMA), identical global_step, matching loss/accuracy
    records -- across several launches (the epoch base advances), an epoch wrap of the
    dataset and a switch back to the pipelined path."""
    from distributedtensorflowexample_amd.train.fused_mlp import FusedMLPTrainer

    nb, lr = 5, 0.3
    p, x, y = _mlp_setup(gpu, B, nb, seed=5)
    p.mul_(0.1)
    tp = FusedMLPTrainer(p, x, y, B, lr)
    tq = FusedMLPTrainer(p, x, y, B, lr)
    assert tq.persistent_ok
    tp.run(7, use_graph=False)
    tp.flush()
    tq.run_persistent(7)
    torch.cuda.synchronize()
    tq.check()
    assert tq.global_step() == tp.global_step() == 7
    assert tq.pos == tp.pos
    d = (tq.params - tp.params).abs().max().item()
    assert d < 1e-6, d
    tp.run(13, use_graph=False)
    for k in (6, 1, 4):
        tq.run_persistent(k)
    tq.run(2, use_graph=False)  # back on the pipelined path
    tp.flush()
    tq.flush()
    torch.cuda.synchronize()
    tq.check()
    assert tq.global_step() == tp.global_step() == 20
    d = (tq.params - tp.params).abs().max().item()
    assert d < 2e-6, d
    assert torch.allclose(tq.stats_range(0, 20), tp.stats_range(0, 20), atol=1e-5)
    # and against the float64 reference
    ref = p.double().cpu()
    xr, yr = x.double().cpu(), y.cpu()
    for s in range(20):
        sl = slice((s % nb) * B, (s % nb + 1) * B)
        g, _, _ = mlp_step.reference_step(ref, xr[sl], yr[sl])
        ref = ref - lr * g
    assert (tq.params.double().cpu() - ref).abs().max().item() < 1e-4


def test_persistent_trainer_long_run(gpu):
    """2000 steps in one persistent launch (epoch parity planes reused 1000 times, 20 dataset
    wraps) track 2000 pipelined steps."""
    from distributedtensorflowexample_amd.data.synthetic import mnist_like_device
    from distributedtensorflowexample_amd.models.mlp import init_params
    from distributedtensorflowexample_amd.train.fused_mlp import FusedMLPTrainer

    p = init_params(gpu, seed=7)
    x, y = mnist_like_device(10000, seed=8, device=gpu)
    tp = FusedMLPTrainer(p, x, y, 100, 0.001)
    tq = FusedMLPTrainer(p, x, y, 100, 0.001)
    tp.run(2000)
    tp.flush()
    tq.run_persistent(2000)
    torch.cuda.synchronize()
    tq.check()
    assert tq.global_step() == tp.global_step() == 2000
    d = (tq.params - tp.params).abs().max().item()
    assert d < 1e-4, d
    assert torch.allclose(tq.stats_range(1000, 2000), tp.stats_range(1000, 2000), atol=1e-4)


def test_persistent_trainer_error_word_drains_and_raises(gpu):
    """A raised error word (what a timed-out hand-off leaves) makes every wait of the next
    persistent launch give up after a few polls: the grid drains quickly and check() raises."""
    import time

    from distributedtensorflowexample_amd.data.synthetic import mnist_like_device
    from distributedtensorflowexample_amd.models.mlp import init_params
    from distributedtensorflowexample_amd.train.fused_mlp import FusedMLPTrainer

    p = init_params(gpu, seed=9)
    x, y = mnist_like_device(1000, seed=9, device=gpu)
    tr = FusedMLPTrainer(p, x, y, 100, 0.01)
    tr.run_persistent(5)
    torch.cuda.synchronize()
    tr.check()
    tr._ll[-32] = 1  # the sticky error word
    t0 = time.perf_counter()
    tr.run_persistent(200, timeout_s=0.5)
    torch.cuda.synchronize()
    assert time.perf_counter() - t0 < 10.0
    with pytest.raises(RuntimeError):
        tr.check()


@pytest.mark.parametrize("locking", [False, True])
def test_gpu_param_store_kernels(gpu, locking):
    """GPU parameter store primitives (csrc/kernels/gpu_ps.*) against a float64 reference:
    pull into a local replica, ApplyGradientDescent (plain lock-free RMW, or f32 atomics with
    use_locking), global_step fetch-add returning the old value, host read / write."""
    from distributedtensorflowexample_amd.ops._ext import hip, stream_handle

    n = mlp_step.NPARAM
    st = hip().GpuParamStore(gpu.index or 0, n, True)
    try:
        p0 = _rand(n, dev="cpu", seed=11)
        g = _rand(n, dev=gpu, seed=12)
        st.write(p0.data_ptr(), 0, n * 4)
        s = stream_handle(gpu)
        for _ in range(3):
            st.push_apply(g.data_ptr(), 0.25, locking, s)
        local = torch.zeros(n, device=gpu)
        st.pull(local.data_ptr(), s)
        torch.cuda.synchronize()
        ref = p0.double() - 3 * 0.25 * g.double().cpu()
        assert (local.double().cpu() - ref).abs().max().item() < 1e-5
        back = torch.empty(n)
        st.read(back.data_ptr(), 0, n * 4)
        assert torch.equal(back, local.cpu())
        assert st.fetch_add(0, 1, s) == 0
        assert st.fetch_add(0, 5, s) == 1
        assert st.fetch_add(0, 0, s) == 6
        rec = torch.tensor([1.5, 0.25], device=gpu)
        old, vals = st.fetch_add_read(0, 1, s, rec.data_ptr(), 2)
        assert old == 6 and vals == [1.5, 0.25] and st.fetch_add(0, 0, s) == 7
    finally:
        st.close()
