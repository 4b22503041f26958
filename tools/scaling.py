"""Scaling curve of the headline benchmark: runs ``bench.py`` at several GPU counts on
one node (N = 1 directly, N > 1 under ``torch.distributed.run``, one process per GPU)
and writes one JSON line per N plus the weak-scaling efficiency
``value(N) / (N * value(1))`` (samples/sec and scaling efficiency).

    python tools/scaling.py --gpus 1 2 4 8 --steps 20000 --warmup 2000 \
        --out profiles/scaling.jsonl [-- extra bench.py args]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def bench_cmd(n, steps, warmup, extra):
    args = [os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", str(steps),
            "--warmup", str(warmup)] + list(extra)
    if n == 1:
        return [sys.executable] + args
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            "--nproc-per-node", str(n), "--master-addr", "127.0.0.1",
            "--master-port", str(_free_port())] + args


def run_one(n, steps, warmup, extra, timeout):
    """One bench run (a child process: nothing here touches the GPU); its JSON line."""
    out = subprocess.run(bench_cmd(n, steps, warmup, extra), capture_output=True, text=True,
                         timeout=timeout, cwd=ROOT)
    for line in reversed(out.stdout.splitlines()):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    raise RuntimeError("bench.py at N=%d printed no result (rc %d):\n%s" % (
        n, out.returncode, (out.stderr or "")[-2000:]))


def efficiency(results):
    """Attach weak-scaling efficiency relative to the N = 1 result (if present)."""
    base = next((r for r in results if r["n_gpus"] == 1), None)
    for r in results:
        r["scaling_efficiency"] = (round(r["value"] / (r["n_gpus"] * base["value"]), 4)
                                   if base else None)
    return results


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=20000)
    ap.add_argument("--warmup", type=int, default=2000)
    ap.add_argument("--timeout", type=float, default=900.0)
    ap.add_argument("--out", default=None, help="JSON-lines output file")
    a, extra = ap.parse_known_args()
    if extra and extra[0] == "--":
        extra = extra[1:]
    results = [run_one(n, a.steps, a.warmup, extra, a.timeout) for n in a.gpus]
    results = efficiency(results)
    lines = [json.dumps(r) for r in results]
    if a.out:
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + "\n")
    for r in results:
        print("N=%d  %14.1f %s  %.3f ms/step  efficiency %s  (%s)" % (
            r["n_gpus"], r["value"], r["unit"], r["ms_per_step"], r["scaling_efficiency"],
            r["config"].get("comm")))


if __name__ == "__main__":
    main()
