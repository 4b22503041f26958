"""Probe: which 3-rank MLP DP engine deviates (run under torch.multiprocessing, one GPU).

Each repetition trains fresh trainers of three engines -- fused LL push (exchange in the
wgrad kernel), all-reduce over the xGMI flag protocol, all-reduce over LL push -- for 40
steps from the same start and prints max |difference| between every pair per rank.
"""
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def worker(rank, world, port, reps):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from distributedtensorflowexample_amd.data.synthetic import mnist_like_device
    from distributedtensorflowexample_amd.models.mlp import init_params
    from distributedtensorflowexample_amd.parallel.xgmi import XgmiComm
    from distributedtensorflowexample_amd.train.fused_mlp import FusedMLPTrainer

    dev = torch.device("cuda:0")
    params = init_params(dev, seed=7)
    x, y = mnist_like_device(2000, seed=50 + rank, device=dev)
    fc = XgmiComm(rank, world, mlp_step.XG_SLOT_WORDS, device=dev, key="p/fused",
                  protocol="push")
    c_flag = XgmiComm(rank, world, params.numel(), device=dev, key="p/flag", protocol="flag")
    c_push = XgmiComm(rank, world, params.numel(), device=dev, key="p/push", protocol="push")
    for rep in range(reps):
        tf = FusedMLPTrainer(params, x, y, 100, 0.05, world_size=world, fused_comm=fc)
        ta = FusedMLPTrainer(params, x, y, 100, 0.05, world_size=world, allreduce=c_flag.allreduce_sum_)
        tb = FusedMLPTrainer(params, x, y, 100, 0.05, world_size=world, allreduce=c_push.allreduce_sum_)
        for t in (tf, ta, tb):
            t.run(7, use_graph=False)
            t.run(33, use_graph=True)
        for c in (fc, c_flag, c_push):
            c.check()
        pf, pa, pb = tf.flush(), ta.flush(), tb.flush()
        d = lambda u, v: float((u - v).abs().max())  # noqa: E731
        print("rep %d rank %d fused-flag %.3g fused-push %.3g flag-push %.3g" % (
            rep, rank, d(pf, pa), d(pf, pb), d(pa, pb)), flush=True)
        dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(worker, args=(world, port, reps), nprocs=world)
