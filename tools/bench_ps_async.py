"""Reference-equivalent baseline: async parameter-server SGD on MI355X.

Runs the reference's topology (1 ps + N workers sharing the GPU(s), per-step
pull 318 KB / push 318 KB + remote apply / fetch_add global_step) through
``main.py`` and the launcher, with the reference's hyper-parameters, and
reports cluster samples/sec = speed (global steps/sec, worker.py:144-146)
x batch_size -- exactly what the reference prints.

    python tools/bench_ps_async.py --num_workers 2 --steps 20000
    python tools/bench_ps_async.py --num_workers 2 --steps 20000 --ps_device gpu
"""
import argparse
import glob
import json
import os
import re
import statistics
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedtensorflowexample_amd.launch import launch_ps  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num_workers", type=int, default=2)
    ap.add_argument("--num_gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20000)
    ap.add_argument("--batch_size", type=int, default=100)
    ap.add_argument("--log_every", type=int, default=1000)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--base_port", type=int, default=24222)
    ap.add_argument("--ps_device", choices=["cpu", "gpu"], default="cpu",
                    help="cpu: the reference's TCP parameter server; gpu: variables in the "
                         "chief's GPU-resident store (parallel/gpu_ps.py)")
    ap.add_argument("--rpc", choices=["fused", "separate"], default="fused",
                    help="fused: push + step + next pull in one pipelined round trip per ps "
                         "task; separate: the reference's three round trips per step")
    ap.add_argument("--cpu_affinity", choices=["numa", "none"], default="numa",
                    help="numa: every cluster process on one NUMA node's CPUs (main.py flag)")
    a = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="psbench")
    import resource
    import time

    ru0, t0 = resource.getrusage(resource.RUSAGE_CHILDREN), time.perf_counter()
    rc = launch_ps(a.num_workers, a.num_gpus, None, 1, cpu=a.cpu, base_port=a.base_port,
                   log_dir=os.path.join(tmp, "logs"), quiet=True, timeout=1800,
                   extra=["--training_steps", str(a.steps), "--log_every", str(a.log_every),
                          "--eval_every", str(10 ** 9), "--logdir", os.path.join(tmp, "m"),
                          "--save_model_secs", "1e9", "--save_summaries_secs", "1e9",
                          "--batch_size", str(a.batch_size), "--ps_device", a.ps_device,
                          "--ps_fused_rpc=%s" % ("true" if a.rpc == "fused" else "false"),
                          "--cpu_affinity", a.cpu_affinity])
    wall = time.perf_counter() - t0
    ru1 = resource.getrusage(resource.RUSAGE_CHILDREN)
    cpu_s = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
    quota = None  # the cgroup's CPU allotment (cgroup v2 cpu.max: "quota period")
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    speeds = []
    for p in glob.glob(os.path.join(tmp, "logs", "worker*.log")):
        for m in re.finditer(r"step: (\d+)\t\| cost: [^|]+\| speed: ([0-9.eE+-]+)step/sec",
                             open(p).read()):
            if int(m.group(1)) > 2 * a.log_every:  # skip warm-up prints
                speeds.append(float(m.group(2)))
    if not speeds:
        print(json.dumps({"error": "no speed prints", "rc": rc}))
        return 1
    sps = statistics.median(speeds)
    print(json.dumps({"metric": "samples/sec (cluster) MNIST MLP async PS (reference semantics)",
                      "value": round(sps * a.batch_size, 1), "unit": "samples/sec",
                      "global_steps_per_sec": round(sps, 1), "num_workers": a.num_workers,
                      "num_gpus": a.num_gpus, "device": "cpu" if a.cpu else "MI355X",
                      "ps_device": a.ps_device, "rpc": a.rpc, "cpu_affinity": a.cpu_affinity,
                      "steps": a.steps, "rc": rc, "n_speed_samples": len(speeds),
                      # CPU time of the whole cluster over its wall time (ps + workers, start
                      # to exit): the CPUs it kept busy, beside the cgroup's allotment
                      "cluster_cpu_seconds": round(cpu_s, 1), "wall_seconds": round(wall, 1),
                      "cpus_busy": round(cpu_s / wall, 2) if wall > 0 else None,
                      "cgroup_cpus": quota}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
