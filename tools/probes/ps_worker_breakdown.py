"""Where an async-PS worker step goes (one GPU worker, in-process C++ ps on localhost):
host-timed phases of Worker's hot loop -- next_batch, local forward/backward (batch H2D,
kernels, TF-layout gradient D2H), the pipelined push + step + pull RPC, the pulled
parameters' H2D + layout conversion, the per-step summary.  Prints medians in us.

    python tools/probes/ps_worker_breakdown.py [--steps 3000]
"""
import argparse
import json
import os
import socket
import statistics
import sys
import tempfile
import time
import types

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributedtensorflowexample_amd.cluster import Server  # noqa: E402
from distributedtensorflowexample_amd.data.mnist import read_data_sets  # noqa: E402
from distributedtensorflowexample_amd.train.worker import Worker  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--mode", choices=["serial", "pipelined"], default="pipelined")
    a = ap.parse_args()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    spec = {"ps": ["127.0.0.1:%d" % port], "worker": ["127.0.0.1:1"]}
    ps = Server(spec, "ps", 0)
    tmp = tempfile.mkdtemp()
    fl = types.SimpleNamespace(batch_size=100, learning_rate=0.001, training_steps=10 ** 9,
                               logdir=os.path.join(tmp, "m"), log_every=10 ** 9,
                               eval_every=10 ** 9, save_model_secs=1e9, save_summaries_secs=1e9,
                               use_locking=False, seed=0, num_workers=1)
    w = Worker("worker", 0, Server(spec, "worker", 0), fl, device=a.device, log=lambda *_: None)
    data = read_data_sets(seed=0)
    w.store.create()
    w.init_op()
    w.sync_op()
    if a.mode == "serial":  # round-3 loop: every phase on the critical path, in sequence
        keys = ("next_batch", "compute", "push_step_pull", "assign_local", "summary", "total")
    else:  # Worker's loop now: next batch drawn + staged while the ps works
        keys = ("compute", "rpc_begin", "stage_next", "rpc_end", "assign_local", "summary",
                "total")
    t = {k: [] for k in keys}
    nxt = None
    for i in range(a.steps):
        if a.mode == "serial":
            t0 = time.perf_counter()
            bx, by = data.train.next_batch(100)
            t1 = time.perf_counter()
            grads, cost, acc = w.compute(bx, by)
            t2 = time.perf_counter()
            step, vals = w.store.push_step_pull(grads, w.lr, False, w.step_name)
            t3 = time.perf_counter()
            w._assign_local(vals)
            if w.device.type == "cuda":
                torch.cuda.synchronize()
            t4 = time.perf_counter()
            w.summary_writer.add_scalars({"loss": cost, "accuracy": acc}, step)
            t5 = time.perf_counter()
            ds = (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t5 - t0)
        else:
            t0 = time.perf_counter()
            if nxt is None:
                bx, by = data.train.next_batch(100)
                grads, cost, acc = w.compute(bx, by)
            else:
                grads, cost, acc = w.compute(*nxt, staged=True)
            t1 = time.perf_counter()
            w.store.push_step_pull_begin(grads, w.lr, False, w.step_name)
            t2 = time.perf_counter()
            nxt = data.train.next_batch(100)
            w.stage(*nxt)
            t3 = time.perf_counter()
            step, vals = w.store.push_step_pull_end()
            t4 = time.perf_counter()
            w._assign_local(vals)
            t5 = time.perf_counter()
            w.summary_writer.add_scalars({"loss": cost, "accuracy": acc}, step)
            t6 = time.perf_counter()
            ds = (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5, t6 - t0)
        if i >= 200:
            for k, d in zip(t, ds):
                t[k].append(d * 1e6)
    out = {k: round(statistics.median(v), 1) for k, v in t.items()}
    out["mode"] = a.mode
    out["steps_per_sec_one_worker"] = round(1e6 / out["total"], 1)
    print(json.dumps(out))
    w.summary_writer.close()
    w.store.close()
    ps.stop()


if __name__ == "__main__":
    main()
