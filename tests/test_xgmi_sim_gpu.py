"""Every xGMI kernel instantiation for world 2..8 (and the flag protocol up to 16),
executed on ONE GPU with simulated peers.

SURVEY §4 ("peer buffers that are local allocations, so the kernel path is identical and
only the pointer origin differs"): ``XgmiComm.with_local_peers`` builds the communicator of
rank r of a W-rank job whose W slot regions are plain allocations on cuda:0.  Before each
launch the test stages, into those regions, exactly the words the W-1 peers would have
written for that round (value + epoch, in the slot of the epoch's parity); the launch then
runs the real kernel of rank r (template instantiation XW = W) and must

  * finish without a timed-out wait (every word it waits for is there),
  * produce the rank-ordered sum / gathered factors / SGD update of a float64 reference
    (exact where the kernel only sums staged f32 values in rank order), and
  * leave in every peer's region exactly the words a real peer would receive.

Two rounds per case cover both slot parities and the device-side epoch advance.  The
rank-to-rank protocol itself (concurrent ranks racing on parities) is exercised by the
multi-process tests in test_xgmi_gpu.py and the shared-GPU rehearsal (scripts/gpu_rehearsal.sh).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

WORLDS = [2, 3, 4, 5, 6, 7, 8]
XG_BLOCKS = 256
MASK32 = 0xFFFFFFFF


def _words(v, epoch):
    """{f32 value, u32 epoch} LL words (int64) of a float32 tensor."""
    bits = v.contiguous().view(torch.int32).to(torch.int64) & MASK32
    return bits | (int(epoch) << 32)


def _vals(w):
    return (w & MASK32).to(torch.int32).view(torch.float32)


def _epochs(w):
    return (w >> 32) & MASK32


def _ordered_sum(vals):
    """float32 sum in rank order starting from 0 -- what every kernel computes."""
    acc = torch.zeros_like(vals[0])
    for v in vals:
        acc = acc + v
    return acc


def _ranks(world):
    return sorted({0, world // 2, world - 1})


# ---------------------------------------------------------------------------------------
# stand-alone all-reduce: LL pull / push / push2 and the flag protocol
# ---------------------------------------------------------------------------------------
def _stage_and_check_allreduce(proto, world, rank, n, dev):
    from distributedtensorflowexample_amd.parallel.xgmi import XgmiComm

    comm, regs = XgmiComm.with_local_peers(rank, world, n, device=dev, protocol=proto)
    S = comm.slot_stride
    g = torch.Generator().manual_seed(100 * world + rank)
    for epoch in (1, 2):  # parity 1 then 0
        par = epoch & 1
        vals = [torch.randn(n, generator=g) * (j + 1) for j in range(world)]
        exp = _ordered_sum(vals)
        vd = [v.to(dev) for v in vals]
        if proto == "ll":  # each rank publishes into its OWN [2][S] slot; readers pull
            for j in range(world):
                if j != rank:
                    regs[j][par * S:par * S + n] = _words(vd[j], epoch)
        elif proto == "push":  # slot(dst, src) = [(par * W + src) * S]
            for j in range(world):
                if j != rank:
                    o = (par * world + j) * S
                    regs[rank][o:o + n] = _words(vd[j], epoch)
        elif proto == "push2":
            shard = (n + world - 1) // world
            s0, s1 = rank * shard, min(n, (rank + 1) * shard)
            for j in range(world):  # reduce-scatter: peers' shares of MY shard
                if j != rank:
                    o = (par * world + j) * S
                    regs[rank][o + s0:o + s1] = _words(vd[j][s0:s1], epoch)
            res = (2 * world + par) * S  # all-gather: owners' sums of THEIR shards
            full = _words(exp.to(dev), epoch)
            regs[rank][res:res + n] = full
        else:  # flag: f32 slots [2][S] + flags [W][XG_BLOCKS] per rank
            for j in range(world):
                if j != rank:
                    regs[j].view(torch.float32)[par * S:par * S + n] = vd[j]
                    fl = regs[rank].view(torch.int32)[2 * S + j * XG_BLOCKS:
                                                      2 * S + (j + 1) * XG_BLOCKS]
                    fl.fill_(epoch)
        t = vd[rank].clone()
        torch.cuda.synchronize()
        comm.allreduce_sum_(t)
        comm.check()
        assert torch.equal(t.cpu(), exp), (proto, world, rank, epoch,
                                           float((t.cpu() - exp).abs().max()))
        # float64 sanity of the same sum
        ref = torch.stack([v.double() for v in vals]).sum(0)
        assert float((t.cpu().double() - ref).abs().max()) <= 1e-5 * float(ref.abs().max())
        # what the peers received
        mine = _words(vd[rank], epoch)
        if proto == "ll":
            assert torch.equal(regs[rank][par * S:par * S + n], mine)
        elif proto == "push":
            for j in range(world):
                if j != rank:
                    o = (par * world + rank) * S
                    assert torch.equal(regs[j][o:o + n], mine), (j, epoch)
        elif proto == "push2":
            shard = (n + world - 1) // world
            for o_rank in range(world):
                if o_rank == rank:
                    continue
                a0, a1 = o_rank * shard, min(n, (o_rank + 1) * shard)
                o = (par * world + rank) * S
                assert torch.equal(regs[o_rank][o + a0:o + a1], mine[a0:a1]), (o_rank, epoch)
                s0, s1 = rank * shard, min(n, (rank + 1) * shard)
                res = (2 * world + par) * S
                assert torch.equal(regs[o_rank][res + s0:res + s1],
                                   _words(exp[s0:s1].to(dev), epoch)), (o_rank, epoch)
        else:
            assert torch.equal(regs[rank].view(torch.float32)[par * S:par * S + n], vd[rank])
            for j in range(world):
                f = regs[j].view(torch.int32)[2 * S + rank * XG_BLOCKS:
                                              2 * S + (rank + 1) * XG_BLOCKS]
                assert bool((f == epoch).all()), (j, epoch)
    comm.destroy()


@pytest.mark.parametrize("world", WORLDS)
@pytest.mark.parametrize("proto", ["ll", "push", "push2"])
def test_ll_allreduce_simulated_peers(gpu, proto, world):
    for rank in _ranks(world):
        for n in (79510, 1021):  # the MLP gradient; a size that is not a multiple of W or 4
            _stage_and_check_allreduce(proto, world, rank, n, gpu)


@pytest.mark.parametrize("world", [2, 3, 5, 8, 12, 16])
def test_flag_allreduce_simulated_peers(gpu, world):
    for rank in _ranks(world):
        _stage_and_check_allreduce("flag", world, rank, 79510, gpu)
        _stage_and_check_allreduce("flag", world, rank, 1021, gpu)


# ---------------------------------------------------------------------------------------
# MLP data-parallel engines: fused (3-launch), fused2 (pipelined), factor, factor2
# ---------------------------------------------------------------------------------------
def _setup(dev, B, seed):
    from distributedtensorflowexample_amd.data.synthetic import mnist_like_device
    from distributedtensorflowexample_amd.models.mlp import init_params
    from distributedtensorflowexample_amd.ops import mlp_step

    p = init_params(dev, seed=seed, stddev=0.3)
    x, y = mnist_like_device(B, seed=seed + 1, device=dev)
    ws = mlp_step.StepWorkspace(B, dev)
    return p, x, y, ws


def _ws_views(ws):
    from distributedtensorflowexample_amd.ops import mlp_step

    B = ws.B
    BP = (B + 15) // 16 * 16
    HP = mlp_step.HP
    # workspace = [slab planes][BP][HP] | hbuf | dz1T | dlT [16][BP] | rowstat [2 BP]; the
    # number of slab planes (the largest K slicing of any first launch) from its size
    planes = (ws.buf.numel() - 2 * BP * HP - 18 * BP) // (BP * HP)
    o = planes * BP * HP
    hbuf = ws.buf[o:o + BP * HP].view(BP, HP)
    o += BP * HP
    dz1T = ws.buf[o:o + HP * BP].view(HP, BP)
    return hbuf, dz1T, BP


def _plain_fwd_head(p, x, y, ws):
    """3-launch layout: K1 (7 slabs) + plain head -> factors of (p, x) in ws."""
    from distributedtensorflowexample_amd.ops._ext import hip, ptr, stream_handle

    h, s = hip(), stream_handle()
    h.mlp_fwd(ptr(p), 0, 0.0, 0, ptr(x), ptr(ws.buf), ws.B, s)
    h.mlp_head(ptr(p), 0, 0.0, 0, ptr(y), ptr(ws.buf), ws.B, s)


def _pipelined_fwd_head(p, x, y, ws):
    """Single-GPU pipelined layout: copy-only fwdapply + head2 -> factors of (p, x) in ws."""
    from distributedtensorflowexample_amd.ops._ext import hip, ptr, stream_handle

    h, s = hip(), stream_handle()
    tmp = p.clone()
    h.mlp_fwdapply(ptr(p), ptr(tmp), 0.0, ptr(x), ptr(x), ptr(ws.buf), ptr(ws.ctr), 0,
                   ws.stats_ring, ws.B, 0, s)
    h.mlp_head2(ptr(tmp), ptr(y), ptr(ws.buf), ws.B, s)


def _ref_grad(p, x, y):
    from distributedtensorflowexample_amd.ops import mlp_step

    g, _, _ = mlp_step.reference_step(p.double().cpu(), x.double().cpu(), y.cpu())
    return g


def _ref_dz1(p, x, y):
    from distributedtensorflowexample_amd.ops import mlp_step

    pd, xd = p.double().cpu(), x.double().cpu()
    W1t, b1, W2t, b2 = mlp_step.unflatten(pd)
    h, logits = mlp_step.reference_forward(pd, xd)
    prob = torch.softmax(logits, 1)
    dl = (prob - torch.nn.functional.one_hot(y.cpu().long(), 10).double()) / x.shape[0]
    return ((dl @ W2t) * h * (1 - h))  # [B, H]


def _stage_param_words(comm, regs, peer_vals, epoch, lo, hi):
    """Peers' LL words for parameter offsets [lo, hi) into MY push slots."""
    S, W, r = comm.slot_stride, comm.world_size, comm.rank
    par = epoch & 1
    for q in range(W):
        if q != r:
            o = (par * W + q) * S
            regs[r][o + lo:o + hi] = _words(peer_vals[q][lo:hi].to(regs[r].device), epoch)


def _check_pushed(comm, regs, own_ref, epoch, lo, hi, tol):
    """Every peer received MY words for [lo, hi) in slot (parity, me), with this epoch."""
    S, W, r = comm.slot_stride, comm.world_size, comm.rank
    par = epoch & 1
    for j in range(W):
        if j == r:
            continue
        o = (par * W + r) * S
        w = regs[j][o + lo:o + hi].cpu()
        assert bool((_epochs(w) == epoch).all()), ("epoch", j, epoch)
        err = float((_vals(w).double() - own_ref[lo:hi]).abs().max())
        assert err <= tol, ("pushed value", j, epoch, err)


def _peer_grads(world, rank, seed, scale):
    from distributedtensorflowexample_amd.ops import mlp_step

    g = torch.Generator().manual_seed(seed)
    return [None if q == rank else torch.randn(mlp_step.NPARAM, generator=g) * scale
            for q in range(world)]


def _expected_update(own, peers, rank):
    tot = torch.zeros_like(own)
    for q, v in enumerate(peers):
        tot += own if q == rank else v.double()
    return tot


def _engine_cases():
    cases = [(w, w - 1, 100) for w in WORLDS]
    cases += [(w, 0, 100) for w in (3, 8)]
    cases += [(w, w // 2, 64) for w in (2, 5, 8)]  # generic (NGT = 0) instantiations
    return cases


@pytest.mark.parametrize("world,rank,B", _engine_cases())
def test_fused_wgrad_exchange_simulated_peers(gpu, world, rank, B):
    """mlp_wgrad_kernel<.., XW>: 3-launch fused engine (exchange in the wgrad epilogue)."""
    from distributedtensorflowexample_amd.ops import mlp_step
    from distributedtensorflowexample_amd.parallel.xgmi import XgmiComm

    p, x, y, ws = _setup(gpu, B, 10 * world + rank)
    comm, regs = XgmiComm.with_local_peers(rank, world, mlp_step.NPARAM, device=gpu)
    _plain_fwd_head(p, x, y, ws)
    own = _ref_grad(p, x, y)
    lr = 0.5
    cur = p.double().cpu()
    for epoch in (1, 2):
        peers = _peer_grads(world, rank, 7 * epoch + world, 0.05)
        _stage_param_words(comm, regs, peers, epoch, 0, mlp_step.NPARAM)
        torch.cuda.synchronize()
        comm.mlp_wgrad(p, lr, x, ws)
        comm.check()
        cur = cur - lr * _expected_update(own, peers, rank)
        err = float((p.double().cpu() - cur).abs().max())
        assert err <= 2e-5, (epoch, err)
        _check_pushed(comm, regs, own, epoch, 0, mlp_step.NPARAM, 2e-6)
    assert ws.global_step() == 2
    comm.destroy()


@pytest.mark.parametrize("world,rank,B", _engine_cases())
def test_fused2_fwdapply_exchange_simulated_peers(gpu, world, rank, B):
    """mlp_fwdapply_kernel<NGT, XW>: pipelined fused engine (step t-1's exchange + apply fused
    with step t's forward)."""
    from distributedtensorflowexample_amd.data.synthetic import mnist_like_device
    from distributedtensorflowexample_amd.ops import mlp_step
    from distributedtensorflowexample_amd.ops._ext import hip, ptr, stream_handle
    from distributedtensorflowexample_amd.parallel.xgmi import XgmiComm

    p_old, x_prev, y_prev, ws = _setup(gpu, B, 20 * world + rank)
    x, y = mnist_like_device(B, seed=999 + rank, device=gpu)
    comm, regs = XgmiComm.with_local_peers(rank, world, mlp_step.XG_SLOT_WORDS, device=gpu)
    lr = 0.5
    bufs = [p_old, torch.empty_like(p_old)]
    batches = [(x_prev, y_prev), (x, y)]
    _pipelined_fwd_head(p_old, x_prev, y_prev, ws)
    # W1 travels in the 16-byte pair layout (xg_exchange16); pairs of padding columns / hidden
    # rows do not travel: stage the whole region anyway (a superset), then the real words
    w1map = mlp_step.xg_w1_pair_offsets().to(gpu)
    n1, S = mlp_step.OFF_B1, comm.slot_stride
    reg_lo, reg_hi = mlp_step.XG_W1_BASE, mlp_step.XG_SLOT_WORDS
    cur = 0
    for epoch in (1, 2):
        xp, yp = batches[(epoch - 1) % 2]
        xn, yn = batches[epoch % 2]
        po, pn = bufs[cur], bufs[cur ^ 1]
        own = _ref_grad(po, xp, yp)
        peers = _peer_grads(world, rank, 11 * epoch + world, 0.05)
        _stage_param_words(comm, regs, peers, epoch, n1, mlp_step.NPARAM)  # small: by offset
        par = epoch & 1
        for q in range(world):
            if q != rank:
                o = (par * world + q) * S
                regs[rank][o + reg_lo:o + reg_hi] = _words(torch.zeros(reg_hi - reg_lo,
                                                                        device=gpu), epoch)
                regs[rank][o + w1map] = _words(peers[q][:n1].to(gpu), epoch)
        exp = po.double().cpu() - lr * _expected_update(own, peers, rank)
        torch.cuda.synchronize()
        comm.mlp_fwdapply(po, pn, lr, xp, xn, ws, True)
        hip().mlp_head2(ptr(pn), ptr(yn), ptr(ws.buf), ws.B, stream_handle(), mlp_step.XG_SLABS)
        comm.check()
        err = float((pn.double().cpu() - exp).abs().max())
        assert err <= 2e-5, (epoch, err)
        _check_pushed(comm, regs, own, epoch, n1, mlp_step.NPARAM, 2e-6)
        dead = torch.ones(reg_hi - reg_lo, dtype=torch.bool)
        dead[w1map.cpu() - reg_lo] = False
        for j in range(world):  # my W1 words reached every peer, in the pair layout
            if j != rank:
                pad = regs[j][(par * world + rank) * S + reg_lo:(par * world + rank) * S + reg_hi]
                assert bool((_epochs(pad.cpu()[dead]) == 0).all())  # padding pairs never sent
                w = regs[j][(par * world + rank) * S + w1map].cpu()
                assert bool((_epochs(w) == epoch).all()), ("epoch", j, epoch)
                assert float((_vals(w).double() - own[:n1]).abs().max()) <= 2e-6
        # step t's forward ran on the UPDATED parameters
        hbuf, _, _ = _ws_views(ws)
        h_ref, _ = mlp_step.reference_forward(pn.double().cpu(), xn.double().cpu())
        herr = float((hbuf[:B, :100].double().cpu() - h_ref).abs().max())
        assert herr <= 1e-4, (epoch, herr)
        cur ^= 1
    assert ws.global_step() == 2
    comm.destroy()


@pytest.mark.parametrize("nslab", [7, 28])
@pytest.mark.parametrize("world,rank,B", _engine_cases())
def test_factor_head_allgather_simulated_peers(gpu, world, rank, B, nslab):
    """mlp_head_kernel<.., XW, NSLAB>: all-gather of the backprop factors dz1 into dz1A."""
    from distributedtensorflowexample_amd.ops import mlp_step
    from distributedtensorflowexample_amd.ops._ext import hip, ptr, stream_handle
    from distributedtensorflowexample_amd.parallel.xgmi import XgmiComm

    p, x, y, ws = _setup(gpu, B, 30 * world + rank)
    comm, regs = XgmiComm.with_local_peers(rank, world, mlp_step.NPARAM, device=gpu)
    BP = (B + 15) // 16 * 16
    HP = mlp_step.HP
    plane = HP * BP
    dz1A = torch.zeros(world, BP, HP, device=gpu)  # [rank][batch row][hidden]
    own = _ref_dz1(p, x, y)  # [B, H]
    S, par_w = comm.slot_stride, world
    g = torch.Generator().manual_seed(5 + world)
    for epoch in (1, 2):
        par = epoch & 1
        peer = {}
        for q in range(world):
            if q == rank:
                continue
            v = torch.zeros(BP, HP)  # the slot's word layout: row * HP + hidden
            v[:B, :100] = torch.randn(B, 100, generator=g)
            peer[q] = v
            o = (par * par_w + q) * S
            regs[rank][o:o + plane] = _words(v.reshape(-1).to(gpu), epoch)
        torch.cuda.synchronize()
        if nslab == 7:
            hip().mlp_fwd(ptr(p), 0, 0.0, 0, ptr(x), ptr(ws.buf), ws.B, stream_handle())
        else:
            tmp = p.clone()  # (a first launch with the factor engines' 28-slice layout)
            hip().mlp_fwdapply(ptr(p), ptr(tmp), 0.0, ptr(x), ptr(x), ptr(ws.buf), ptr(ws.ctr),
                               0, ws.stats_ring, ws.B, 0, stream_handle(), ks=nslab)
        comm.mlp_head(p, y, ws, dz1A, nslab=nslab)
        comm.check()
        got = dz1A.cpu()
        for q in range(world):
            if q == rank:
                err = float((got[q, :B, :100].double() - own).abs().max())
                assert err <= 1e-5, (epoch, err)
            else:
                assert torch.equal(got[q, :B, :100], peer[q][:B, :100]), (epoch, q)
        # every peer received my factors for (row < B, j < 100)
        for j in range(world):
            if j == rank:
                continue
            o = (par * world + rank) * S
            w = regs[j][o:o + plane].cpu().view(BP, HP)[:B, :100]
            assert bool((_epochs(w) == epoch).all()), (j, epoch)
            assert float((_vals(w).double() - own).abs().max()) <= 1e-5
    comm.destroy()


def _factor_inputs(world, rank, B, dev, seed):
    from distributedtensorflowexample_amd.data.synthetic import mnist_like_device
    from distributedtensorflowexample_amd.ops import mlp_step

    BP = (B + 15) // 16 * 16
    x_all = torch.stack([mnist_like_device(B, seed=seed + q, device=dev)[0]
                         for q in range(world)]).contiguous()
    g = torch.Generator().manual_seed(seed)
    dz1A = torch.zeros(world, BP, mlp_step.HP)  # [rank][batch row][hidden], row-major
    dz1A[:, :B, :100] = torch.randn(world, B, 100, generator=g) * 0.01
    return x_all, dz1A.to(dev)


def _global_w1_grad(dz1A, x_all, B):
    W = x_all.shape[0]
    g = torch.zeros(100, 784, dtype=torch.float64)
    for q in range(W):
        g += dz1A[q, :B, :100].double().cpu().t() @ x_all[q].double().cpu()
    return g.reshape(-1)


@pytest.mark.parametrize("world,rank,B", _engine_cases())
def test_factor_wgrad_simulated_peers(gpu, world, rank, B):
    """mlp_wgrad_factor_kernel<XW, NGT>: global dW1 from every rank's factors and batch, small
    parameters exchanged (LL push)."""
    from distributedtensorflowexample_amd.ops import mlp_step
    from distributedtensorflowexample_amd.parallel.xgmi import XgmiComm

    p, _, y, ws = _setup(gpu, B, 40 * world + rank)
    x_all, dz1A = _factor_inputs(world, rank, B, gpu, 77 + world)
    x = x_all[rank]
    comm, regs = XgmiComm.with_local_peers(rank, world, mlp_step.NPARAM, device=gpu)
    _plain_fwd_head(p, x, y, ws)
    own = _ref_grad(p, x, y)
    gW1 = _global_w1_grad(dz1A, x_all, B)
    lr = 0.5
    cur = p.double().cpu()
    lo = mlp_step.OFF_B1
    for epoch in (1, 2):
        peers = _peer_grads(world, rank, 13 * epoch + world, 0.05)
        _stage_param_words(comm, regs, peers, epoch, lo, mlp_step.NPARAM)
        torch.cuda.synchronize()
        comm.mlp_wgrad_factor(p, lr, x, x_all.stride(0), dz1A, ws)
        comm.check()
        upd = _expected_update(own, peers, rank)
        upd[:lo] = gW1
        cur = cur - lr * upd
        err = float((p.double().cpu() - cur).abs().max())
        assert err <= 2e-5, (epoch, err)
        _check_pushed(comm, regs, own, epoch, lo, mlp_step.NPARAM, 2e-6)
    assert ws.global_step() == 2
    comm.destroy()


@pytest.mark.parametrize("world,rank,B", _engine_cases())
def test_factor2_fwdapply_simulated_peers(gpu, world, rank, B):
    """mlp_fwdapply_factor_kernel<XW, NGT>: pipelined factor engine (global W1 update of step
    t-1 from every rank's factors and previous batch, small parameters exchanged, fused with
    step t's forward)."""
    from distributedtensorflowexample_amd.data.synthetic import mnist_like_device
    from distributedtensorflowexample_amd.ops import mlp_step
    from distributedtensorflowexample_amd.ops._ext import hip, ptr, stream_handle
    from distributedtensorflowexample_amd.parallel.xgmi import XgmiComm

    p_old, _, y_prev, ws = _setup(gpu, B, 50 * world + rank)
    x_all, dz1A = _factor_inputs(world, rank, B, gpu, 91 + world)
    x_prev = x_all[rank]
    x, y = mnist_like_device(B, seed=555 + rank, device=gpu)
    comm, regs = XgmiComm.with_local_peers(rank, world, mlp_step.NPARAM, device=gpu)
    lr = 0.5
    lo = mlp_step.OFF_B1
    _pipelined_fwd_head(p_old, x_prev, y_prev, ws)
    own = _ref_grad(p_old, x_prev, y_prev)
    gW1 = _global_w1_grad(dz1A, x_all, B)
    p_new = torch.empty_like(p_old)
    peers = _peer_grads(world, rank, 17 + world, 0.05)
    _stage_param_words(comm, regs, peers, 1, lo, mlp_step.NPARAM)
    torch.cuda.synchronize()
    comm.mlp_fwdapply_factor(p_old, p_new, lr, x_prev, x, x_all.stride(0), dz1A, ws, True)
    hip().mlp_head2(ptr(p_new), ptr(y), ptr(ws.buf), ws.B, stream_handle(), mlp_step.FACTOR_SLABS)
    comm.check()
    upd = _expected_update(own, peers, rank)
    upd[:lo] = gW1
    exp = p_old.double().cpu() - lr * upd
    err = float((p_new.double().cpu() - exp).abs().max())
    assert err <= 2e-5, err
    _check_pushed(comm, regs, own, 1, lo, mlp_step.NPARAM, 2e-6)
    hbuf, _, _ = _ws_views(ws)
    h_ref, _ = mlp_step.reference_forward(p_new.double().cpu(), x.double().cpu())
    assert float((hbuf[:B, :100].double().cpu() - h_ref).abs().max()) <= 1e-4
    # second round (parity 0): the factors of (p_new, x) now sit in ws
    own2 = _ref_grad(p_new, x, y)
    x_all2, dz1A2 = _factor_inputs(world, rank, B, gpu, 191 + world)
    x_all2[rank] = x
    gW1b = _global_w1_grad(dz1A2, x_all2, B)
    peers2 = _peer_grads(world, rank, 19 + world, 0.05)
    _stage_param_words(comm, regs, peers2, 2, lo, mlp_step.NPARAM)
    p3 = torch.empty_like(p_old)
    torch.cuda.synchronize()
    comm.mlp_fwdapply_factor(p_new, p3, lr, x_all2[rank], x, x_all2.stride(0), dz1A2, ws, True)
    comm.check()
    upd2 = _expected_update(own2, peers2, rank)
    upd2[:lo] = gW1b
    exp2 = p_new.double().cpu() - lr * upd2
    assert float((p3.double().cpu() - exp2).abs().max()) <= 2e-5
    _check_pushed(comm, regs, own2, 2, lo, mlp_step.NPARAM, 2e-6)
    assert ws.global_step() == 2
    comm.destroy()


def test_timeout_when_a_peer_word_is_missing(gpu):
    """A word a peer never wrote is a bounded wait, reported through the error word (no hang)."""
    from distributedtensorflowexample_amd.parallel.xgmi import XgmiComm

    world, rank, n = 8, 3, 4096
    comm, regs = XgmiComm.with_local_peers(rank, world, n, device=gpu, protocol="push",
                                           timeout_s=0.05)
    S = comm.slot_stride
    for j in range(world):
        if j not in (rank, 6):  # peer 6 never publishes
            o = (1 * world + j) * S
            regs[rank][o:o + n] = _words(torch.ones(n, device=gpu), 1)
    t = torch.ones(n, device=gpu)
    comm.allreduce_sum_(t)
    assert comm.failed()
    comm.destroy()


# ---------------------------------------------------------------------------------------
# bandwidth-mode two-shot all-reduce (large buckets): f32 payload + per-block release flags
# ---------------------------------------------------------------------------------------
def _bw_check(world, rank, n, S_numel, dev):
    from distributedtensorflowexample_amd.parallel.xgmi import XgmiComm

    comm, regs = XgmiComm.with_local_peers(rank, world, S_numel, device=dev, protocol="bw")
    S = comm.slot_stride
    CS = ((S + world - 1) // world + 3) // 4 * 4
    cs = ((n + world - 1) // world + 3) // 4 * 4
    flags0 = 2 * world * CS + 2 * S  # int32 index of the flag array
    m = [max(0, min(cs, n - c * cs)) for c in range(world)]
    g = torch.Generator().manual_seed(31 * world + rank + n)
    for epoch in (1, 2, 3):
        par = epoch & 1
        vals = [torch.randn(n, generator=g) * (j + 1) for j in range(world)]
        exp = _ordered_sum(vals)
        vd = [v.to(dev) for v in vals]
        ed = exp.to(dev)
        f = regs[rank].view(torch.float32)
        fl = regs[rank].view(torch.int32)
        for j in range(world):
            if j == rank:
                continue
            o = (par * world + j) * CS
            f[o:o + m[rank]] = vd[j][rank * cs:rank * cs + m[rank]]
            fl[flags0 + (0 * world + j) * XG_BLOCKS:flags0 + (0 * world + j + 1) * XG_BLOCKS] = epoch
            fl[flags0 + (1 * world + j) * XG_BLOCKS:flags0 + (1 * world + j + 1) * XG_BLOCKS] = epoch
        ag = 2 * world * CS + par * S
        for c in range(world):
            if c != rank:
                f[ag + c * cs:ag + c * cs + m[c]] = ed[c * cs:c * cs + m[c]]
        t = vd[rank].clone()
        torch.cuda.synchronize()
        comm.allreduce_sum_(t)
        comm.check()
        assert torch.equal(t.cpu(), exp), (world, rank, n, epoch,
                                           float((t.cpu() - exp).abs().max()))
        for q in range(world):  # what every peer received from me
            if q == rank:
                continue
            fq, flq = regs[q].view(torch.float32), regs[q].view(torch.int32)
            o = (par * world + rank) * CS
            assert torch.equal(fq[o:o + m[q]], vd[rank][q * cs:q * cs + m[q]]), (q, epoch)
            assert torch.equal(fq[ag + rank * cs:ag + rank * cs + m[rank]],
                               ed[rank * cs:rank * cs + m[rank]]), (q, epoch)
            for ph in (0, 1):
                a = flags0 + (ph * world + rank) * XG_BLOCKS
                assert bool((flq[a:a + XG_BLOCKS] == epoch).all()), (q, ph, epoch)
    comm.destroy()


@pytest.mark.parametrize("world", WORLDS)
def test_bw_allreduce_simulated_peers(gpu, world):
    for rank in _ranks(world):
        # a BERT-layer-sized bucket, a size that is not a multiple of W * 4 or of the block
        # split, and a bucket smaller than the communicator's capacity
        for n, cap in ((7 * 1024 * 1024 + 13, 7 * 1024 * 1024 + 13), (100003, 100003),
                       (5000, 1 << 20)):
            _bw_check(world, rank, n, cap, gpu)


def _bw_shard_check(world, rank, n, dev, dtype):
    """The bw kernel's halves (ZeRO-1): reduce-scatter -- chunk r of g becomes the rank-ordered
    sum of every rank's chunk r, and each peer's receive slot holds my share of its chunk;
    all-gather -- my chunk lands in every peer's gather region, and the peers' chunks staged in
    mine land in g.  bf16 all-gathers travel as f32 words."""
    from distributedtensorflowexample_amd.parallel.xgmi import XgmiComm

    words = n if dtype == torch.float32 else n // 2
    comm, regs = XgmiComm.with_local_peers(rank, world, words, device=dev, protocol="bw")
    S = comm.slot_stride
    CS = ((S + world - 1) // world + 3) // 4 * 4
    cs = words // world
    flags0 = 2 * world * CS + 2 * S
    g = torch.Generator().manual_seed(17 * world + rank + n)
    f = regs[rank].view(torch.float32)
    fl = regs[rank].view(torch.int32)
    ops = ("rs", "ag", "rs", "ag") if dtype == torch.float32 else ("ag", "ag")
    for epoch, op in enumerate(ops, 1):  # (the device epoch advances once per call)
        par = epoch & 1
        ph = 0 if op == "rs" else 1
        for j in range(world):
            if j != rank:
                fl[flags0 + (ph * world + j) * XG_BLOCKS:flags0 + (ph * world + j + 1) * XG_BLOCKS] = epoch
        if op == "rs":
            vals = [torch.randn(n, generator=g) * (j + 1) for j in range(world)]
            exp = _ordered_sum([v[rank * cs:(rank + 1) * cs] for v in vals])
            for j in range(world):
                if j != rank:
                    o = (par * world + j) * CS
                    f[o:o + cs] = vals[j][rank * cs:(rank + 1) * cs].to(dev)
            t = vals[rank].to(dev)
            torch.cuda.synchronize()
            comm.reduce_scatter(t[rank * cs:(rank + 1) * cs], t)
            comm.check()
            assert torch.equal(t[rank * cs:(rank + 1) * cs].cpu(), exp), (world, rank, epoch)
            for q in range(world):
                if q != rank:
                    o = (par * world + rank) * CS
                    assert torch.equal(regs[q].view(torch.float32)[o:o + cs].cpu(),
                                       vals[rank][q * cs:(q + 1) * cs]), (q, epoch)
        else:
            full = (torch.randn(n, generator=g) * 3).to(dtype)
            fw = full.view(torch.float32) if dtype != torch.float32 else full
            ag = 2 * world * CS + par * S
            for c in range(world):
                if c != rank:
                    f[ag + c * cs:ag + (c + 1) * cs] = fw[c * cs:(c + 1) * cs].to(dev)
            t = torch.zeros(n, device=dev, dtype=dtype)
            k = n // world
            t[rank * k:(rank + 1) * k] = full[rank * k:(rank + 1) * k].to(dev)
            torch.cuda.synchronize()
            comm.all_gather(t, t[rank * k:(rank + 1) * k])
            comm.check()
            assert torch.equal(t.cpu(), full), (world, rank, epoch)
            for q in range(world):
                if q != rank:
                    assert torch.equal(regs[q].view(torch.float32)[ag + rank * cs:ag + (rank + 1) * cs].cpu(),
                                       fw[rank * cs:(rank + 1) * cs]), (q, epoch)
    comm.destroy()


@pytest.mark.parametrize("world", WORLDS)
def test_bw_reduce_scatter_all_gather_simulated_peers(gpu, world):
    for rank in _ranks(world):
        for n in (64 * world * 1000, 64 * world * 3):
            _bw_shard_check(world, rank, n, gpu, torch.float32)
            _bw_shard_check(world, rank, n, gpu, torch.bfloat16)


def _pair_owner(words, world):
    """Owner rank of a word of the 16-byte pair layout in the pair two-shot exchange
    (xg_exchange2p): pair (eslot, sp, lane) is owned by (lane // 16 + 4 sp) % world."""
    from distributedtensorflowexample_amd.ops import mlp_step

    pi = (words - mlp_step.XG_W1_BASE) // 2
    lane, sp = pi % 64, (pi // 64) % 2
    return (lane // 16 + 4 * sp) % world


@pytest.mark.parametrize("world,rank", [(2, 1), (3, 2), (4, 1), (5, 0), (6, 4), (7, 6), (8, 7),
                                        (8, 3)])
def test_fused2_two_shot_exchange_simulated_peers(gpu, world, rank):
    """mlp_fwdapply_kernel<7, XW, false, true>: the W1 tiles' exchange as reduce-scatter +
    all-gather of 16-byte word pairs (xg_exchange2p; owned pairs: gather + rank-ordered sum +
    broadcast; the others: push to the owner, then take its sums); small parameters one-shot."""
    from distributedtensorflowexample_amd.data.synthetic import mnist_like_device
    from distributedtensorflowexample_amd.ops import mlp_step
    from distributedtensorflowexample_amd.ops._ext import hip, ptr, stream_handle
    from distributedtensorflowexample_amd.parallel.xgmi import XgmiComm

    B = 100
    p_old, x_prev, y_prev, ws = _setup(gpu, B, 60 * world + rank)
    x, y = mnist_like_device(B, seed=777 + rank, device=gpu)
    comm, regs = XgmiComm.with_local_peers(rank, world, mlp_step.engine_slot_words("fused2x"),
                                           device=gpu)
    comm.two_shot = True
    S = comm.slot_stride
    n1 = mlp_step.OFF_B1
    w1map = mlp_step.xg_w1_pair_offsets()
    owner = _pair_owner(w1map, world)
    mine = owner == rank
    reg = torch.arange(mlp_step.XG_W1_BASE, mlp_step.XG_SLOT_WORDS)
    dead = torch.ones(reg.numel(), dtype=torch.bool)
    dead[w1map - mlp_step.XG_W1_BASE] = False  # words of no W1 element (padding pairs)
    w1g, mg = w1map.to(gpu), mine.to(gpu)
    lr = 0.5
    bufs = [p_old, torch.empty_like(p_old)]
    batches = [(x_prev, y_prev), (x, y)]
    _pipelined_fwd_head(p_old, x_prev, y_prev, ws)
    g = torch.Generator().manual_seed(world * 31 + rank)
    cur = 0
    for epoch in (1, 2):
        par = epoch & 1
        xp, yp = batches[(epoch - 1) % 2]
        xn, yn = batches[epoch % 2]
        po, pn = bufs[cur], bufs[cur ^ 1]
        own = _ref_grad(po, xp, yp)
        peers = _peer_grads(world, rank, 23 * epoch + world, 0.05)
        # small parameters: one-shot slots, every peer
        _stage_param_words(comm, regs, peers, epoch, n1, mlp_step.NPARAM)
        # W1, owned pairs: the peers' contributions (padding words: zeros of this epoch);
        # not owned: the owner's (arbitrary) sums in my result region
        for q in range(world):
            if q != rank:
                o = (par * world + q) * S
                regs[rank][o + reg] = _words(torch.zeros(reg.numel(), device=gpu), epoch)
                regs[rank][o + w1g[mg]] = _words(peers[q][:n1].to(gpu)[mg], epoch)
        owners_sum = torch.randn(n1, generator=g) * 0.07
        res = (2 * world + par) * S
        regs[rank][res + reg] = _words(torch.zeros(reg.numel(), device=gpu), epoch)
        regs[rank][res + w1g[~mg]] = _words(owners_sum.to(gpu)[~mg], epoch)
        tot = _expected_update(own, peers, rank)
        exp = po.double().cpu() - lr * tot
        exp[:n1][~mine] = po.double().cpu()[:n1][~mine] - lr * owners_sum.double()[~mine]
        torch.cuda.synchronize()
        comm.mlp_fwdapply(po, pn, lr, xp, xn, ws, True)
        hip().mlp_head2(ptr(pn), ptr(yn), ptr(ws.buf), ws.B, stream_handle(), mlp_step.XG_SLABS)
        comm.check()
        err = float((pn.double().cpu() - exp).abs().max())
        assert err <= 2e-5, (epoch, err)
        # pushes: my pairs went to their owner only; my sums of the owned pairs to every
        # peer's result region
        for d in range(world):
            if d == rank:
                continue
            o = (par * world + rank) * S
            to_d = owner == d
            wv = regs[d][o + w1g].cpu()
            assert bool((_epochs(wv[to_d]) == epoch).all()), ("contribution epoch", d)
            assert float((_vals(wv[to_d]).double() - own[:n1][to_d]).abs().max()) <= 2e-6
            rv = regs[d][res + w1g].cpu()
            assert bool((_epochs(rv[mine]) == epoch).all()), ("result epoch", d)
            got = _vals(rv[mine]).double()
            assert float((got - tot[:n1][mine]).abs().max()) <= 2e-5
            # pairs of padding columns / hidden rows never travel (neither pushed nor broadcast)
            rr = regs[d][res + reg].cpu()
            cc = regs[d][o + reg].cpu()
            assert bool((_epochs(rr[dead]) == 0).all()), ("result padding", d)
            assert bool((_epochs(cc[dead]) == 0).all()), ("contribution padding", d)
        _check_pushed(comm, regs, own, epoch, n1, mlp_step.NPARAM, 2e-6)
        cur ^= 1
    comm.destroy()


@pytest.mark.parametrize("world", [2, 8])
def test_simulated_peers_comm_shape(gpu, world):
    """parallel.xgmi.SimulatedPeersComm (tools/probes/dp_sim.py): the real bandwidth-mode
    two-shot of rank 0 over never-writing simulated peers -- its own chunk comes back as the
    rank-ordered sum (own + zeros), every other chunk as zeros; buckets above max_numel go in
    pieces; the flags were pre-raised, so nothing waits or fails."""
    from distributedtensorflowexample_amd.parallel.xgmi import SimulatedPeersComm

    n, cap = 10_000, 4_096
    c = SimulatedPeersComm(world, cap, device=gpu)
    g = torch.randn(n, device=gpu)
    ref = g.clone()
    c.allreduce_sum_(g)
    torch.cuda.synchronize()
    assert not c.failed()
    for lo in range(0, n, cap):
        piece, want = g[lo:lo + cap], ref[lo:lo + cap]
        cs = ((piece.numel() + world - 1) // world + 3) // 4 * 4
        assert torch.equal(piece[:cs], want[:cs])
        assert not piece[cs:].any()
    c.destroy()
