"""Cluster launcher: replaces the reference's tmux scripts (run_*_gpu.sh).

The reference opens one tmux window per task and starts
``CUDA_VISIBLE_DEVICES= python main.py --job_name ps`` plus one
``CUDA_VISIBLE_DEVICES=${GPU_ID[i % num_gpus]} python main.py --job_name
worker --task_index i`` per worker (run_single_gpu.sh:17-22).  This launcher
does the same with subprocesses (``HIP_VISIBLE_DEVICES``), writes one log per
task, streams them with a ``[task]`` prefix, waits for the workers, then
stops the parameter servers (the reference's ps never exits).

    python -m distributedtensorflowexample_amd.launch ps --num_workers 2 --num_gpus 1
    python -m distributedtensorflowexample_amd.launch mirrored --nproc 8
    ... -- --training_steps 20000 --learning_rate 0.001   (extra main.py flags)

``mirrored`` spawns one process per GPU with RANK / WORLD_SIZE / LOCAL_RANK /
MASTER_ADDR / MASTER_PORT set (what torch.distributed.run would set).
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAIN = os.path.join(ROOT, "main.py")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _pump(proc, name, logf, quiet):
    for line in iter(proc.stdout.readline, b""):
        logf.write(line)
        logf.flush()
        if not quiet:
            sys.stdout.write("[%s] %s" % (name, line.decode(errors="replace")))
            sys.stdout.flush()


def _cpu_threads(nproc):
    """OMP_NUM_THREADS for one of nproc CPU-device tasks on this host: the user's setting, else
    a fair share of the cores (torch's default of every core per process oversubscribes the
    host nproc-fold and the gloo/TCP tasks stall one another)."""
    return os.environ.get("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 1) // max(1, nproc))))


class Cluster:
    def __init__(self, log_dir, quiet=False):
        self.log_dir = log_dir
        self.quiet = quiet
        os.makedirs(log_dir, exist_ok=True)
        self.procs = {}
        self._threads = []

    def spawn(self, name, args, env_extra):
        env = dict(os.environ)
        env.update(env_extra)
        env.setdefault("PYTHONUNBUFFERED", "1")
        logf = open(os.path.join(self.log_dir, name + ".log"), "wb")
        p = subprocess.Popen([sys.executable, MAIN] + args, env=env, stdout=subprocess.PIPE,
                             stderr=subprocess.STDOUT, cwd=ROOT)
        t = threading.Thread(target=_pump, args=(p, name, logf, self.quiet), daemon=True)
        t.start()
        self.procs[name] = p
        self._threads.append(t)
        return p

    def wait(self, names, timeout=None, fail_fast=False, poll=0.1, grace=10.0):
        """Wait for ``names``; {name: returncode, None if still running at ``timeout``}.

        ``fail_fast`` (sync DP): every task is polled, and as soon as one exits non-zero the
        others are stopped (SIGTERM, SIGKILL after ``grace`` s) -- a synchronous job cannot
        make progress without every rank, and a rank blocked in a collective with a dead
        peer would otherwise hold the launcher until ``timeout``."""
        t0 = time.time()
        if not fail_fast:
            rc = {}
            for n in names:
                left = None if timeout is None else max(0.1, timeout - (time.time() - t0))
                try:
                    rc[n] = self.procs[n].wait(left)
                except subprocess.TimeoutExpired:
                    rc[n] = None
            return rc
        while True:
            rc = {n: self.procs[n].poll() for n in names}
            failed = [n for n in names if rc[n] not in (None, 0)]
            if failed:
                alive = [n for n in names if rc[n] is None]
                if alive:
                    print("launch: %s exited with %s; stopping %s" % (
                        failed[0], rc[failed[0]], ", ".join(alive)), file=sys.stderr, flush=True)
                    self.terminate(alive, grace)
                return {n: self.procs[n].poll() for n in names}
            if all(v is not None for v in rc.values()):
                return rc
            if timeout is not None and time.time() - t0 > timeout:
                return rc
            time.sleep(poll)

    def terminate(self, names, grace=10.0):
        for n in names:
            p = self.procs[n]
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        t0 = time.time()
        for n in names:
            p = self.procs[n]
            try:
                p.wait(max(0.1, grace - (time.time() - t0)))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        for t in self._threads:
            t.join(timeout=2)


def launch_ps(num_workers=2, num_gpus=1, gpu_ids=None, num_ps=1, extra=(), log_dir="launch_logs",
              base_port=12222, timeout=None, quiet=False, cpu=False):
    """1..num_ps ps tasks + num_workers workers; returns {task: returncode}."""
    gpu_ids = list(gpu_ids) if gpu_ids else list(range(num_gpus))
    common = ["--num_workers", str(num_workers), "--num_gpus", str(num_gpus), "--num_ps",
              str(num_ps), "--base_port", str(base_port)] + list(extra)
    if cpu:
        common += ["--device", "cpu"]
    cl = Cluster(log_dir, quiet)
    ps_names = []
    for i in range(num_ps):
        n = "ps%d" % i
        cl.spawn(n, ["--job_name", "ps", "--task_index", str(i)] + common,
                 {"HIP_VISIBLE_DEVICES": "", "CUDA_VISIBLE_DEVICES": ""})
        ps_names.append(n)
    w_names = []
    for i in range(num_workers):
        n = "worker%d" % i
        env = {} if cpu else {"HIP_VISIBLE_DEVICES": str(gpu_ids[i % len(gpu_ids)])}
        if cpu:
            env.update({"HIP_VISIBLE_DEVICES": "", "CUDA_VISIBLE_DEVICES": "",
                        "OMP_NUM_THREADS": _cpu_threads(num_workers)})
        cl.spawn(n, ["--job_name", "worker", "--task_index", str(i)] + common, env)
        w_names.append(n)
    try:
        rc = cl.wait(w_names, timeout)
    finally:
        cl.terminate([n for n in cl.procs if cl.procs[n].poll() is None])
    return rc


def launch_mirrored(nproc=1, extra=(), log_dir="launch_logs", timeout=None, quiet=False):
    port = _free_port()
    cl = Cluster(log_dir, quiet)
    names = []
    ex = list(extra)
    cpu = "--device" in ex and ex.index("--device") + 1 < len(ex) and ex[ex.index("--device") + 1] == "cpu"
    for r in range(nproc):
        n = "rank%d" % r
        env = {"RANK": str(r), "WORLD_SIZE": str(nproc), "LOCAL_RANK": str(r),
               "LOCAL_WORLD_SIZE": str(nproc), "MASTER_ADDR": "127.0.0.1",
               "MASTER_PORT": str(port)}
        if cpu:
            env["OMP_NUM_THREADS"] = _cpu_threads(nproc)
        cl.spawn(n, ["--strategy", "mirrored"] + ex, env)
        names.append(n)
    try:
        rc = cl.wait(names, timeout, fail_fast=True)
    finally:
        cl.terminate([n for n in cl.procs if cl.procs[n].poll() is None])
    return rc


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    extra = []
    if "--" in argv:
        i = argv.index("--")
        argv, extra = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawTextHelpFormatter)
    sub = ap.add_subparsers(dest="mode", required=True)
    p = sub.add_parser("ps", help="async parameter-server cluster (the reference's mode)")
    p.add_argument("--num_workers", type=int, default=2)
    p.add_argument("--num_gpus", type=int, default=1)
    p.add_argument("--gpu_ids", type=str, default="", help="comma list, default 0..num_gpus-1")
    p.add_argument("--num_ps", type=int, default=1)
    p.add_argument("--base_port", type=int, default=12222)
    p.add_argument("--cpu", action="store_true", help="CPU-only workers (plumbing config)")
    m = sub.add_parser("mirrored", help="sync data parallel, one process per GPU")
    m.add_argument("--nproc", type=int, default=1)
    for q in (p, m):
        q.add_argument("--log_dir", default="launch_logs")
        q.add_argument("--timeout", type=float, default=None)
        q.add_argument("--quiet", action="store_true")
    a = ap.parse_args(argv)
    if a.mode == "ps":
        ids = [int(x) for x in a.gpu_ids.split(",") if x != ""] or None
        rc = launch_ps(a.num_workers, a.num_gpus, ids, a.num_ps, extra, a.log_dir, a.base_port,
                       a.timeout, a.quiet, a.cpu)
    else:
        rc = launch_mirrored(a.nproc, extra, a.log_dir, a.timeout, a.quiet)
    bad = {k: v for k, v in rc.items() if v != 0}
    if bad:
        print("launch: tasks failed: %s" % bad, file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
