"""Training loops on the GPU: async-PS worker (fused kernels) and sync-DP trainer."""
import types

import pytest

pytestmark = pytest.mark.gpu


def _flags(tmp_path, **kw):
    d = dict(batch_size=100, learning_rate=0.01, training_steps=200, logdir=str(tmp_path / "m"),
             log_every=100, eval_every=100, save_model_secs=1000.0, save_summaries_secs=1000.0,
             use_locking=False, seed=0, device="cuda")
    d.update(kw)
    return types.SimpleNamespace(**d)


@pytest.fixture(scope="module")
def mnist():
    from distributedtensorflowexample_amd.data.mnist import read_data_sets

    return read_data_sets(seed=0)


def test_ps_worker_gpu_matches_cpu_math(gpu, tmp_path, mnist):
    from distributedtensorflowexample_amd.cluster import Server
    from distributedtensorflowexample_amd.train.worker import Worker

    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    spec = {"ps": ["127.0.0.1:%d" % port], "worker": ["127.0.0.1:1"]}
    ps = Server(spec, "ps", 0)
    try:
        logs = []
        w = Worker("worker", 0, Server(spec, "worker", 0), _flags(tmp_path), device="cuda",
                   log=logs.append)
        assert w.use_fused
        hist = w.learn(mnist)
        assert len(hist) == 201 and hist[-1][0] == 200
        assert hist[-1][1] < hist[0][1]  # loss went down
        assert any(l.startswith("test accuracy") for l in logs)
        # the GPU fused gradient equals the CPU reference on the same params/batch
        bx, by = mnist.train.next_batch(100)
        w.sync_op()
        g_gpu, l_gpu, _ = w.compute(bx, by)
        w.use_fused = False
        g_cpu, l_cpu, _ = w.compute(bx, by)
        for k in g_gpu:
            assert (g_gpu[k] - g_cpu[k]).abs().max().item() < 1e-4 * max(1, g_cpu[k].abs().max())
    finally:
        ps.stop()


def test_mirrored_gpu_single_rank_with_restore(gpu, tmp_path, mnist):
    from distributedtensorflowexample_amd.train.mirrored_mlp import train_mirrored
    from distributedtensorflowexample_amd.train.saver import latest_checkpoint, load_checkpoint

    fl = _flags(tmp_path, training_steps=1100, learning_rate=0.1, eval_every=1100)
    logs = []
    hist, p = train_mirrored(fl, mnist, log=logs.append)
    assert hist[-1][0] == 1100
    acc = float([l for l in logs if l.startswith("test accuracy")][-1].split()[-1])
    assert acc > 0.3, logs  # learns real digits from the synthetic train set
    ck = latest_checkpoint(fl.logdir)
    assert int(load_checkpoint(ck)["global/global_step"]) == 1100
    # resume: chief restores and continues from 1100 to 1200
    fl2 = _flags(tmp_path, training_steps=1200, learning_rate=0.1, eval_every=10 ** 9)
    hist2, _ = train_mirrored(fl2, mnist, log=logs.append)
    assert hist2[0][0] > 1100 and hist2[-1][0] == 1200


def test_mirrored_gpu_periodic_checkpoints_do_not_perturb_training(gpu, tmp_path, mnist):
    """Checkpoints requested every 20 ms by the Supervisor's timer are taken by the training
    loop between chunks (never by the timer thread, which must not flush the fused
    trainer): training ends bit-identical to a run without periodic saves."""
    import glob
    import time

    import torch

    from distributedtensorflowexample_amd.train import saver as saver_mod
    from distributedtensorflowexample_amd.train.mirrored_mlp import train_mirrored

    out = {}
    for tag, secs in (("quiet", 1000.0), ("busy", 0.02)):
        fl = _flags(tmp_path / tag, training_steps=3000, log_every=50, eval_every=10 ** 9,
                    save_model_secs=secs, check_replicas_every=100)
        orig = saver_mod.Saver.save
        n_saves, threads = [0], set()

        def counting(self, *a, **k):
            n_saves[0] += 1
            threads.add(__import__("threading").current_thread().name)
            time.sleep(0.005)  # give the timer a chance to fire again mid-run
            return orig(self, *a, **k)

        saver_mod.Saver.save = counting
        try:
            hist, p = train_mirrored(fl, mnist, log=lambda *_: None)
        finally:
            saver_mod.Saver.save = orig
        assert hist[-1][0] == 3000
        out[tag] = (p.cpu(), n_saves[0], threads)
    assert out["busy"][1] > out["quiet"][1] >= 1, (out["busy"][1], out["quiet"][1])
    assert out["busy"][2] == {"MainThread"}, out["busy"][2]
    assert torch.equal(out["busy"][0], out["quiet"][0])
