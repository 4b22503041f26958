"""Native RCCL communicator on one GPU (1-rank communicator) incl. hipGraph capture."""
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm(gpu):
    from distributedtensorflowexample_amd.parallel.comm import NativeComm

    c = NativeComm(0, 1, store=dist.HashStore())
    yield c
    c.destroy()


def test_allreduce_identity_and_graph(comm, gpu):
    t = torch.arange(1000, device=gpu, dtype=torch.float32)
    ref = t.clone()
    comm.allreduce_sum_(t)
    torch.cuda.synchronize()
    assert torch.equal(t, ref)
    # capture an allreduce + a kernel in one graph
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        t.mul_(2.0)
        comm.allreduce_sum_(t)
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(t, ref * 4)


def test_collectives_one_rank(comm, gpu):
    x = torch.randn(64, device=gpu)
    out = torch.empty_like(x)
    comm.all_gather(out, x)
    comm.reduce_scatter(out, x)
    comm.broadcast_(x, 0)
    torch.cuda.synchronize()
    assert torch.equal(out, x)
    for dt in (torch.float32, torch.bfloat16):
        a = torch.randn(4, 96, device=gpu).to(dt)
        b = torch.empty_like(a)
        comm.all_to_all(b, a)
        torch.cuda.synchronize()
        assert torch.equal(a, b)


def test_ulysses_and_zero1_over_rccl(comm, gpu):
    """Ulysses SP with its all-to-alls as real RCCL calls (1-rank communicator) and ZeRO-1
    driven by the native communicator give the single-device results (at world 1 the
    ZeRO-1 exchanges reduce to copies)."""
    from distributedtensorflowexample_amd.ops import transformer as T
    from distributedtensorflowexample_amd.optim import AdamOptimizer
    from distributedtensorflowexample_amd.parallel.mirrored import DistributedDataParallel
    from distributedtensorflowexample_amd.parallel.sequence import ulysses_attention
    from distributedtensorflowexample_amd.parallel.sharded import ShardedOptimizer

    B, S, NH = 2, 128, 12
    qkv = (torch.randn(B * S, 3 * NH * 64, device=gpu) * 0.5).to(torch.bfloat16)
    o_ref, _ = T.attn_fwd(qkv, B, S, NH)
    o = ulysses_attention(qkv, comm, B, S, NH)
    torch.cuda.synchronize()
    assert torch.equal(o, o_ref)

    lin_a, lin_b = torch.nn.Linear(64, 48).to(gpu), torch.nn.Linear(64, 48).to(gpu)
    lin_b.load_state_dict(lin_a.state_dict())
    da = DistributedDataParallel(lin_a, comm)
    db = DistributedDataParallel(lin_b, comm, shard=True)
    oa, ob = AdamOptimizer(0.01), ShardedOptimizer(AdamOptimizer(0.01), db)
    x = torch.randn(32, 64, device=gpu)
    for _ in range(3):
        for m, d in ((lin_a, da), (lin_b, db)):
            d.reset()
            m(x).square().mean().backward()
        da.finish()
        oa.apply_gradients([(da.flat_grad, da.flat)])
        ob.step()
    torch.cuda.synchronize()
    assert (lin_a.weight - lin_b.weight).abs().max().item() < 1e-6


def test_dp_trainer_with_native_comm_matches_direct(comm, gpu):
    """Sync-DP step (grad -> RCCL -> deferred apply) == fused single-GPU step."""
    from distributedtensorflowexample_amd.data.synthetic import mnist_like_device
    from distributedtensorflowexample_amd.models.mlp import init_params
    from distributedtensorflowexample_amd.train.fused_mlp import FusedMLPTrainer

    p = init_params(gpu, seed=5) * 0.1
    x, y = mnist_like_device(1000, seed=1, device=gpu)
    a = FusedMLPTrainer(p, x, y, 100, 0.5, allreduce=comm.allreduce_sum_, world_size=1)
    b = FusedMLPTrainer(p, x, y, 100, 0.5)
    a.run(37)
    b.run(37)
    a.flush()
    b.flush()  # (the pipelined single-GPU step defers its last update too)
    torch.cuda.synchronize()
    assert a.global_step() == b.global_step() == 37
    assert (a.params - b.params).abs().max().item() < 1e-5
