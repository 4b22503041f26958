"""Capacity of the TCP parameter server alone (no GPU work): N client processes each loop
push(318 KB gradient) + apply + global_step += 1 + pull(318 KB) as ONE pipelined round trip
(``PSClient.push_step_pull``, the async-PS worker's per-step RPC) against one in-process
``PSServer`` holding the reference MLP's variables.  Reports round trips per second (= global
steps/s the ps + localhost TCP could sustain if the workers' compute were free), so the async
cluster's scaling with workers (tools/bench_ps_async.py) can be split into "ps/transport
bound" and "worker/GPU-sharing bound".

    python tools/probes/ps_capacity.py --clients 1,2,4,8 --secs 3
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SPECS = [("global/dense/kernel", [784, 100]), ("global/dense/bias", [100]),
         ("global/dense_1/kernel", [100, 10]), ("global/dense_1/bias", [10])]


def node_cpus(n=None):
    """CPUs of the NUMA node this process runs on (all allowed CPUs if sysfs says nothing)."""
    allowed = sorted(os.sched_getaffinity(0))
    here = os.sched_getcpu() if hasattr(os, "sched_getcpu") else allowed[0]
    try:
        for d in sorted(os.listdir("/sys/devices/system/node")):
            if not d.startswith("node"):
                continue
            cl = open("/sys/devices/system/node/%s/cpulist" % d).read().strip()
            cpus = set()
            for part in cl.split(","):
                lo, _, hi = part.partition("-")
                cpus.update(range(int(lo), int(hi or lo) + 1))
            if here in cpus:
                sel = [c for c in allowed if c in cpus]
                return sel[:n] if n else sel
    except OSError:
        pass
    return allowed[:n] if n else allowed


def client(addr, secs, q, start, cpus=None):
    if cpus:
        os.sched_setaffinity(0, cpus)
    from distributedtensorflowexample_amd.ops import host

    c = host().PSClient([addr], 30.0, 0.0)
    hs = [c.lookup(n, 0) for n, _ in SPECS]
    step = c.lookup("global/global_step", 0)
    grads = [np.random.default_rng(1).standard_normal(int(np.prod(s))).astype(np.float32) * 1e-3
             for _, s in SPECS]
    pulls = [np.empty(int(np.prod(s)), np.float32) for _, s in SPECS]
    gp, gs = [g.ctypes.data for g in grads], [g.nbytes for g in grads]
    pp, ps = [p.ctypes.data for p in pulls], [p.nbytes for p in pulls]
    start.wait()
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < secs:
        c.push_step_pull(hs, gp, gs, 1e-3, False, step, 1, hs, pp, ps)
        n += 1
    q.put((n, time.perf_counter() - t0))
    c.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", default="1,2,4,8")
    ap.add_argument("--secs", type=float, default=3.0)
    ap.add_argument("--port", type=int, default=25333)
    ap.add_argument("--pin", choices=["none", "server", "all", "compact"], default="none",
                    help="server: the ps process (its connection threads) on the CPUs of one NUMA "
                         "node; all: the clients too")
    ap.add_argument("--pin_cpus", type=int, default=16)
    a = ap.parse_args()
    node_all = node_cpus() if a.pin != "none" else None
    cpus = node_cpus(a.pin_cpus) if a.pin in ("server", "all") else None
    if a.pin == "compact":  # main.py --cpu_affinity numa: server 8 cores, client i 2 after them
        cpus = node_all[:8]
    if cpus:
        os.sched_setaffinity(0, cpus)
    from distributedtensorflowexample_amd.ops import host

    srv = host().PSServer("127.0.0.1", a.port)
    srv.start()
    addr = "127.0.0.1:%d" % srv.port
    c = host().PSClient([addr], 30.0, 0.0)
    for n, s in SPECS:
        h = c.create(n, "float32", s, 0)
        v = np.zeros(int(np.prod(s)), np.float32)
        c.assign(h, v.ctypes.data, v.nbytes)
    h = c.create("global/global_step", "int64", [], 0)
    z = np.zeros(1, np.int64)
    c.assign(h, z.ctypes.data, 8)
    out = {"cpus": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "pin": a.pin,
           "pinned_cpus": cpus, "rows": []}
    ctx = mp.get_context("spawn")
    for k in [int(v) for v in a.clients.split(",")]:
        q, start = ctx.Queue(), ctx.Event()
        def ccpus(i):
            if a.pin == "all":
                return cpus
            if a.pin == "compact":
                return [node_all[(8 + 2 * i + j) % len(node_all)] for j in range(2)]
            return None

        ps = [ctx.Process(target=client, args=(addr, a.secs, q, start, ccpus(i))) for i in range(k)]
        for p in ps:
            p.start()
        time.sleep(2.0)  # imports + connects
        start.set()
        res = [q.get(timeout=a.secs + 60) for _ in ps]
        for p in ps:
            p.join()
        rate = sum(n / t for n, t in res)
        out["rows"].append({"clients": k, "round_trips_per_s": round(rate, 1),
                            "per_client_us": round(1e6 * k / rate, 1)})
        print(json.dumps(out["rows"][-1]), file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)
    c.shutdown_server(0)
    srv.stop()


if __name__ == "__main__":
    main()
