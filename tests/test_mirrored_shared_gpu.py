"""``--strategy mirrored`` with two ranks sharing ONE GPU (DTFX_SHARED_GPU=1: an xGMI-IPC
communicator stands in for RCCL, which refuses two ranks on one device).

Covers the advisor's round-2 finding: periodic checkpoints (chief only), the chief-only
test-accuracy eval and the replica check must never start a peer exchange on one rank while
the pipelined exchange engines (fused2 / factor2) hold a pending update.  With a 50 ms
save_model_secs the chief checkpoints at nearly every chunk boundary; the replicas must stay
bit-identical (``check_replicas_every``) and end identical to the all-reduce engine's run.
"""
import os
import socket
import types

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, logdir, engine, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank), DTFX_SHARED_GPU="1",
                          DTFX_MLP_ENGINE=engine)
        import torch
        import torch.distributed as dist

        from distributedtensorflowexample_amd.data.mnist import read_data_sets
        from distributedtensorflowexample_amd.train import saver as saver_mod
        from distributedtensorflowexample_amd.train.mirrored_mlp import train_mirrored

        fl = types.SimpleNamespace(batch_size=100, learning_rate=0.05, training_steps=1200,
                                   logdir=logdir, log_every=50, eval_every=400,
                                   save_model_secs=0.05, save_summaries_secs=1000.0,
                                   use_locking=False, seed=0, device="cuda",
                                   check_replicas_every=100)
        saves = [0]
        orig = saver_mod.Saver.save

        def counting(self, *a, **k):
            saves[0] += 1
            return orig(self, *a, **k)

        saver_mod.Saver.save = counting
        logs = []

        def log(line):  # ~20 ms per chunk on the chief: the 50 ms save timer fires mid-run
            import time

            logs.append(line)
            time.sleep(0.02)

        hist, p = train_mirrored(fl, read_data_sets(seed=0), log=log)
        chk = p.double().sum().reshape(1).cpu()
        ref = chk.clone()
        dist.broadcast(ref, 0)
        ok = hist[-1][0] == 1200 and torch.equal(chk, ref)
        if rank == 0:
            ok &= saves[0] >= 3 and any(l.startswith("test accuracy") for l in logs)
        q.put((rank, ok, "step %d saves %d sum %.9g" % (hist[-1][0], saves[0], float(chk)),
               p.cpu()))
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        import traceback

        q.put((rank, False, traceback.format_exc()[-2000:], None))


def _run(engine, tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port, world = _port(), 2
    logdir = str(tmp_path / engine / "m")
    procs = [ctx.Process(target=_worker, args=(r, world, port, logdir, engine, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=400) for _ in range(world)]
    for p in procs:
        p.join(60)
    for r, ok, msg, _ in res:
        assert ok, (engine, r, msg)
    return res[0][3]


def test_mirrored_two_ranks_checkpoints_with_pipelined_exchange_engines(gpu, tmp_path):
    base = _run("allreduce", tmp_path)
    for engine in ("fused2", "factor2"):
        p = _run(engine, tmp_path)
        err = float((p - base).abs().max())
        assert err <= 1e-4 * (1.0 + float(base.abs().max())), (engine, err)
