"""Fault injection in a live async parameter-server cluster (1 ps + 2 workers, localhost CPU:
BASELINE config 1), the failures the reference leaves to TF's Supervisor (worker.py:107-118,
main.py:51-55,66-70):

* a worker is SIGKILLed mid-run and restarted: it looks the variables up again, passes the
  ready wait (they are initialised) and continues the SHARED global_step;
* the ps is SIGKILLed: every worker exits non-zero within a bounded time (a lost connection
  is a ConnectionError, not a retry or a hang), and a restarted cluster's chief restores the
  last checkpoint and finishes the run from there;
* the ps hangs (SIGSTOP): with ``--ps_timeout_secs`` the workers give up and exit non-zero.
"""
import os
import re
import signal
import socket
import subprocess
import sys
import time

import pytest

from distributedtensorflowexample_amd.train.saver import latest_checkpoint, load_checkpoint

pytestmark = pytest.mark.slow
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STEP = re.compile(r"^step: (\d+)\t")


def _base_port(n=3):
    """A free run of n consecutive ports (ps, worker0, worker1)."""
    for _ in range(50):
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            p = s.getsockname()[1]
        if p + n >= 65535:
            continue
        ok = True
        for q in range(p, p + n):
            with socket.socket() as s:
                try:
                    s.bind(("127.0.0.1", q))
                except OSError:
                    ok = False
                    break
        if ok:
            return p
    raise RuntimeError("no free port range")


class _Cluster:
    def __init__(self, tmp_path, port, extra):
        self.tmp, self.port, self.extra = tmp_path, port, list(extra)
        self.procs = {}
        self.n = 0

    def start(self, job, task):
        name = "%s%d" % (job, task)
        self.n += 1
        log = str(self.tmp / ("%s.%d.log" % (name, self.n)))
        args = [sys.executable, os.path.join(ROOT, "main.py"), "--job_name", job,
                "--task_index", str(task), "--num_workers", "2", "--base_port", str(self.port)]
        if job == "worker":
            args += self.extra
        env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="",
                   PYTHONUNBUFFERED="1", OMP_NUM_THREADS="2")
        p = subprocess.Popen(args, stdout=open(log, "w"), stderr=subprocess.STDOUT, cwd=ROOT,
                             env=env)
        self.procs[name] = (p, log)
        return p, log

    def kill_all(self):
        for p, _ in self.procs.values():
            if p.poll() is None:
                p.kill()
                p.wait(30)


def _steps(log):
    with open(log) as f:
        return [int(m.group(1)) for m in map(STEP.match, f) if m]


def _wait_for(cond, timeout, what):
    t0 = time.time()
    while time.time() - t0 < timeout:
        v = cond()
        if v:
            return v
        time.sleep(0.1)
    raise AssertionError("timed out waiting for " + what)


def _tail(log):
    with open(log) as f:
        return f.read()[-3000:]


def test_worker_killed_and_restarted_rejoins_shared_global_step(tmp_path):
    total = 40000
    cl = _Cluster(tmp_path, _base_port(), [
        "--device", "cpu", "--training_steps", str(total), "--logdir", str(tmp_path / "m"),
        "--log_every", "200", "--eval_every", str(10 ** 9), "--learning_rate", "0.01",
        "--save_model_secs", "1000"])
    try:
        cl.start("ps", 0)
        w0, log0 = cl.start("worker", 0)
        w1, log1 = cl.start("worker", 1)
        # both workers are in the hot loop, the shared step is well past startup
        _wait_for(lambda: _steps(log0) and _steps(log1) and max(_steps(log0) + _steps(log1))
                  >= 4000, 120, "both workers training")
        w1.send_signal(signal.SIGKILL)
        assert w1.wait(30) == -signal.SIGKILL
        killed_at = max(_steps(log0) + _steps(log1))
        # the chief alone keeps advancing the shared counter meanwhile
        _wait_for(lambda: max(_steps(log0)) > killed_at + 400, 60, "chief progress")
        w1b, log1b = cl.start("worker", 1)
        assert w1b.wait(240) == 0, _tail(log1b)
        assert w0.wait(240) == 0, _tail(log0)
        after = _steps(log1b)
        # the restarted worker looked the variables up, passed the ready wait and continued
        # the SHARED global step: it never starts over at 0
        assert after and min(after) > killed_at, (killed_at, after[:3])
        final = max(_steps(log0) + after)
        assert final >= total - 200, final
    finally:
        cl.kill_all()


def test_ps_death_ends_workers_and_chief_restores_on_restart(tmp_path):
    logdir = str(tmp_path / "m")
    common = ["--device", "cpu", "--logdir", logdir, "--log_every", "200",
              "--eval_every", str(10 ** 9), "--learning_rate", "0.01", "--save_model_secs", "0.5"]
    port = _base_port()
    cl = _Cluster(tmp_path, port, common + ["--training_steps", str(10 ** 7)])
    try:
        ps, _ = cl.start("ps", 0)
        w0, log0 = cl.start("worker", 0)
        w1, log1 = cl.start("worker", 1)
        ck = _wait_for(lambda: (lambda c: c if c and int(load_checkpoint(c)["global/global_step"])
                                > 1000 else None)(latest_checkpoint(logdir)), 120,
                       "a checkpoint past step 1000")
        ps.send_signal(signal.SIGKILL)
        ps.wait(30)
        t0 = time.time()
        rc0, rc1 = w0.wait(60), w1.wait(60)
        # a lost ps ends every worker with an error, promptly (no retry loop, no hang)
        assert rc0 not in (0, None) and rc1 not in (0, None), (rc0, rc1)
        assert time.time() - t0 < 30
        assert "ConnectionError" in _tail(log0) or "PSConnectionLost" in _tail(log0), _tail(log0)
        ck = latest_checkpoint(logdir)
        saved = int(load_checkpoint(ck)["global/global_step"])
        # restart the whole cluster: the chief restores the last checkpoint (restore-or-init)
        total = saved + 3000
        cl2 = _Cluster(tmp_path, port, common + ["--training_steps", str(total)])
        cl2.n = 10
        try:
            cl2.start("ps", 0)
            v0, lg0 = cl2.start("worker", 0)
            v1, lg1 = cl2.start("worker", 1)
            assert v0.wait(240) == 0, _tail(lg0)
            assert v1.wait(240) == 0, _tail(lg1)
            steps = sorted(_steps(lg0) + _steps(lg1))
            assert steps and steps[0] >= saved, (saved, steps[:3])  # resumed, not from 0
            # the resumed run checkpoints past the restored step (periodic saves only, like
            # TF's Supervisor: no final save)
            assert int(load_checkpoint(latest_checkpoint(logdir))["global/global_step"]) > saved
        finally:
            cl2.kill_all()
    finally:
        cl.kill_all()


def test_hung_ps_ends_workers_with_rpc_timeout(tmp_path):
    cl = _Cluster(tmp_path, _base_port(), [
        "--device", "cpu", "--training_steps", str(10 ** 7), "--logdir", str(tmp_path / "m"),
        "--log_every", "200", "--eval_every", str(10 ** 9), "--save_model_secs", "1000",
        "--ps_timeout_secs", "2"])
    try:
        ps, _ = cl.start("ps", 0)
        w0, log0 = cl.start("worker", 0)
        w1, log1 = cl.start("worker", 1)
        _wait_for(lambda: _steps(log0) or _steps(log1), 120, "training")
        ps.send_signal(signal.SIGSTOP)  # alive but silent
        t0 = time.time()
        rc0, rc1 = w0.wait(60), w1.wait(60)
        assert rc0 not in (0, None) and rc1 not in (0, None), (rc0, rc1)
        assert time.time() - t0 < 30
        ps.send_signal(signal.SIGCONT)
    finally:
        cl.kill_all()
