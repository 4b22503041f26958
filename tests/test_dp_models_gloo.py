"""Sync data-parallel BERT / ResNet trainers on CPU with gloo (world_size 2).

Each rank trains on its own data shard; after a few steps every replica must
hold bit-identical parameters, and one DP step must equal a single-process
step whose gradient is the average of the two shards' gradients.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.slow


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _make(kind, comm, rank):
    if kind == "bert":
        from distributedtensorflowexample_amd.models.bert import BertConfig
        from distributedtensorflowexample_amd.train.bert_trainer import BertTrainer

        # (the all-reduce path; the owner-sharded optimizer, the world > 1 default, has its own
        # test below)
        return BertTrainer(BertConfig.tiny(), 2, 32, "cpu", comm=comm, lr=1e-3, data_seed=10 + rank,
                           zero1=False)
    from distributedtensorflowexample_amd.train.resnet_trainer import ResNetTrainer

    return ResNetTrainer(2, "cpu", comm=comm, lr=0.05, image_size=32, stages=[(8, 1, 1), (16, 1, 2)],
                         num_classes=10, data_seed=10 + rank)


def _worker(kind, rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from distributedtensorflowexample_amd.parallel.comm import TorchComm

    tr = _make(kind, TorchComm(), rank)
    tr.run(1)
    g = tr.model.params.grad.clone()  # all-reduced (summed) gradient of step 1
    tr.run(2)
    q.put((rank, tr.model.params.master.numpy().copy(), g.numpy().copy()))  # by value
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["bert", "resnet"])
def test_dp_replicas_identical_and_grad_is_shard_sum(kind):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(kind, r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (torch.from_numpy(m), torch.from_numpy(g)))
               for r, m, g in [q.get(timeout=300) for _ in range(world)])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert torch.equal(res[0][0], res[1][0])          # replicas identical after 3 steps
    # the all-reduced gradient equals the sum of the per-shard single-process gradients
    shard = []
    for r in range(world):
        tr = _make(kind, None, r)
        tr.model.forward_backward(*tr.data[:4], n_valid=tr.data[4]) if kind == "bert" else \
            tr.model.forward_backward(*tr.data)
        shard.append(tr.model.params.grad.clone())
    ref = shard[0] + shard[1]
    assert torch.allclose(res[0][1], ref, atol=1e-5, rtol=1e-4)


def _zero1_worker(rank, world, port, q, zero1, kind="bert"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from distributedtensorflowexample_amd.parallel.comm import TorchComm

    if kind == "bert":
        from distributedtensorflowexample_amd.models.bert import BertConfig
        from distributedtensorflowexample_amd.train.bert_trainer import BertTrainer

        tr = BertTrainer(BertConfig.tiny(), 2, 32, "cpu", comm=TorchComm(), lr=1e-3,
                         data_seed=10 + rank, zero1=zero1)
    else:
        from distributedtensorflowexample_amd.train.resnet_trainer import ResNetTrainer

        tr = ResNetTrainer(2, "cpu", comm=TorchComm(), lr=0.05, image_size=32,
                           stages=[(8, 1, 1), (16, 1, 2)], num_classes=10, data_seed=10 + rank,
                           zero1=zero1)
    tr.run(3)
    tr.sync_params()
    P = tr.model.params
    if kind == "bert":
        sd = {k: v.numpy().copy() for k, v in P.state_dict().items()}
    else:  # by name: the sharded layout pads every bucket to W shards
        sd = {name: P.view(P.master, name).numpy().copy() for name, _, _ in P.layout}
        sd.update({"bf/" + name: P.view(P.bf, name).float().numpy().copy()
                   for name, _, _ in P.layout})
        sd.update({"running/" + n + "/" + str(i): t.numpy().copy()
                   for n, ts in P.running.items() for i, t in enumerate(ts)})
    q.put((rank, sd, P.master.numel(), tr.zero1))
    dist.destroy_process_group()


def _run(world, zero1, kind="bert"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_zero1_worker, args=(r, world, port, q, zero1, kind))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (sd, n, z)) for r, sd, n, z in [q.get(timeout=300) for _ in range(world)])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world", [2, 4])
def test_bert_zero1_matches_replicated_adam(world):
    """Owner-sharded AdamW (reduce-scatter -> AdamW on this rank's shard -> all-gather, the
    reference's apply-once-on-the-owner, worker.py:75-79) against the replicated optimizer over
    3 steps: every parameter to f32 rounding, replicas identical, bucket padding for W shards."""
    sh = _run(world, True)
    rep = _run(world, False)
    assert all(z for _, _, z in sh.values()) and not any(z for _, _, z in rep.values())
    assert sh[0][1] % (64 * world) == 0           # every bucket split into W aligned shards
    for r in range(1, world):                     # replicas identical (sharded)
        for k in sh[0][0]:
            assert (sh[r][0][k] == sh[0][0][k]).all(), (r, k)
    for k, v in rep[0][0].items():                # same trajectory as the replicated AdamW
        d = abs(torch.from_numpy(sh[0][0][k]) - torch.from_numpy(v)).max().item()
        assert d <= 1e-6 + 1e-5 * abs(torch.from_numpy(v)).max().item(), (k, d)


@pytest.mark.parametrize("world", [2, 4])
def test_resnet_zero1_matches_replicated_sgd(world):
    """ResNet owner-sharded momentum SGD (reduce-scatter -> SGD on this rank's shard ->
    all-gather beside the next forward) against the replicated optimizer over 3 steps: every
    parameter, its bf16 working copy and the BatchNorm running statistics to f32 rounding,
    replicas identical, every bucket padded to W aligned shards."""
    sh = _run(world, True, "resnet")
    rep = _run(world, False, "resnet")
    assert all(z for _, _, z in sh.values()) and not any(z for _, _, z in rep.values())
    assert sh[0][1] % (64 * world) == 0
    for r in range(1, world):  # (BatchNorm running statistics are per-rank: local batches)
        for k in sh[0][0]:
            if not k.startswith("running/"):
                assert (sh[r][0][k] == sh[0][0][k]).all(), (r, k)
    for k, v in rep[0][0].items():
        d = abs(torch.from_numpy(sh[0][0][k]) - torch.from_numpy(v)).max().item()
        tol = 1e-6 + 1e-5 * abs(torch.from_numpy(v)).max().item()
        if k.startswith("bf/"):
            tol = 1e-2 * max(1.0, abs(torch.from_numpy(v)).max().item())  # one bf16 ulp
        assert d <= tol, (k, d)
