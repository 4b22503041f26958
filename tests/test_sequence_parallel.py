"""Ulysses sequence parallelism (parallel/sequence.py) on CPU with gloo: attention over a
sequence split across 2 ranks equals single-process attention over the whole sequence,
forward and backward."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.slow

B, S, NH = 2, 16, 4


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs():
    g = torch.Generator().manual_seed(11)
    qkv = (torch.randn(B * S, 3 * NH * 64, generator=g) * 0.5).to(torch.bfloat16)
    dout = torch.randn(B * S, NH * 64, generator=g).to(torch.bfloat16)
    kmask = torch.zeros(B, S)
    kmask[1, S - 5:] = -10000.0  # padded keys in the second sequence
    return qkv, dout, kmask


def _rows(t, rank, world):
    sl = S // world
    return t.view(B, S, -1)[:, rank * sl:(rank + 1) * sl].reshape(B * sl, -1)


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from distributedtensorflowexample_amd.parallel.comm import TorchComm
        from distributedtensorflowexample_amd.parallel.sequence import ulysses_attention

        qkv, dout, kmask = _inputs()
        x = _rows(qkv, rank, world).clone().requires_grad_(True)
        o = ulysses_attention(x, TorchComm(), B, S // world, NH, kmask)
        o.backward(_rows(dout, rank, world))
        # by value: a shared-memory tensor dies with the child before the parent reads it
        q.put((rank, o.detach().float().numpy().copy(), x.grad.float().numpy().copy(), ""))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover - reported through the queue
        import traceback
        q.put((rank, None, None, traceback.format_exc()))


def test_ulysses_matches_full_sequence_attention():
    from distributedtensorflowexample_amd.ops import transformer as T

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
    qkv, dout, kmask = _inputs()
    o_ref, lse = T.attn_fwd(qkv, B, S, NH, kmask)
    dqkv_ref = T.attn_bwd(qkv, o_ref, dout, lse, B, S, NH, kmask)
    for rank, o, g, msg in res:
        assert o is not None, msg
        o, g = torch.from_numpy(o), torch.from_numpy(g)
        assert (o - _rows(o_ref, rank, world).float()).abs().max().item() < 1e-2
        assert (g - _rows(dqkv_ref, rank, world).float()).abs().max().item() < 1e-2


def test_ulysses_rejects_indivisible_heads():
    from distributedtensorflowexample_amd.parallel.sequence import ulysses_attention

    class _C:
        world_size, rank = 3, 0

    with pytest.raises(ValueError):
        ulysses_attention(torch.zeros(B * 4, 3 * NH * 64, dtype=torch.bfloat16), _C(), B, 4, NH)
