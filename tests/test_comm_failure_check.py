"""check_comm_collective: a timed-out xGMI all-reduce on ANY rank stops EVERY
rank at the same step (a gloo collective over the ranks' failed() flags); HybridComm routes on
properties all ranks share."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distributedtensorflowexample_amd.parallel.select import HybridComm, check_comm_collective


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _FakeComm:
    def __init__(self, bad):
        self.bad = bad

    def failed(self):
        return self.bad


def _worker(rank, port, bad_rank, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        check_comm_collective(_FakeComm(rank == bad_rank), "step 7")
        q.put((rank, "ok"))
    except RuntimeError as e:
        q.put((rank, str(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bad_rank", [-1, 0, 1])
def test_failure_flag_is_agreed_by_every_rank(bad_rank):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, port, bad_rank, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(30)
    if bad_rank < 0:
        assert res == {0: "ok", 1: "ok"}
    else:  # both ranks raise, whichever one timed out
        assert all("timed out" in res[r] and "step 7" in res[r] for r in (0, 1)), res


def test_hybrid_routes_on_shared_properties_only():
    class Rec:
        def __init__(self):
            self.calls = []
            self.max_numel = 1 << 20
            self.rank, self.world_size, self.device = 0, 2, None

        def allreduce_sum_(self, t):
            self.calls.append(t.numel())
            return t

        def failed(self):
            return False

    rccl, bw = Rec(), Rec()
    h = HybridComm(rccl, bw, lo=1000)
    h.allreduce_sum_(torch.zeros(4000))        # CPU tensor: never the xGMI kernel
    assert rccl.calls == [4000] and bw.calls == []
    assert h.failed() is False
