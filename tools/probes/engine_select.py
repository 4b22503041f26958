"""Probe: pick_mlp_engine on 2 ranks sharing one GPU, every stage logged to a file.

    python tools/probes/engine_select.py [world] [mode]   -> gpurun_out/engine_select_<rank>.log
"""
import datetime
import os
import socket
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def worker(rank, world, port, mode):
    log = open(os.path.join(ROOT, "gpurun_out", "engine_select_%d.log" % rank), "w")

    def say(*a):
        log.write("%.3f %s\n" % (time.time(), " ".join(str(x) for x in a)))
        log.flush()

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60))
    torch.cuda.set_device(0)
    from distributedtensorflowexample_amd.data.synthetic import mnist_like_device
    from distributedtensorflowexample_amd.models.mlp import init_params
    from distributedtensorflowexample_amd.parallel import select
    from distributedtensorflowexample_amd.parallel.xgmi import XgmiComm
    from distributedtensorflowexample_amd.train import fused_mlp

    dev = torch.device("cuda:0")
    params = init_params(dev, seed=1234)
    n = int(os.environ.get("PROBE_N", "5500"))
    x_all = torch.stack([mnist_like_device(n, seed=100 + q, device=dev)[0]
                         for q in range(world)]).contiguous()
    y = mnist_like_device(n, seed=100 + rank, device=dev)[1]
    ar = XgmiComm(rank, world, params.numel(), device=dev, key="e/ar", protocol="ll")
    say("setup done")
    orig_run = fused_mlp.FusedMLPTrainer.run

    def run(self, steps, use_graph=True):
        say("run", "factor" if self.factor_comm is not None else
            ("fused" if self.fused_comm is not None else "allreduce"),
            "pipelined" if self.pipelined else "", steps, use_graph, "pending", self.pending)
        r = orig_run(self, steps, use_graph)
        torch.cuda.synchronize()
        say("  done")
        return r

    fused_mlp.FusedMLPTrainer.run = run
    kind, c, probe = select.pick_mlp_engine(params, x_all[rank], y, 100, 0.001, ar, world, rank,
                                            dev, mode=mode, x_all=x_all,
                                            time_steps=int(os.environ.get("PROBE_T", "100")))
    say("picked", kind, probe)
    dist.destroy_process_group()


if __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    mode = sys.argv[2] if len(sys.argv) > 2 else "auto"
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(worker, args=(world, port, mode), nprocs=world)
