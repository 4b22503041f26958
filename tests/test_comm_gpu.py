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
