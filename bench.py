#!/usr/bin/env python3
"""Headline benchmark: whole-node samples/sec of the reference's MNIST MLP
trained with synchronous data-parallel SGD on N MI355X (BASELINE.json).

    python bench.py --gpus 1 --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

Config = the reference's (main.py:30-31, worker.py:46-79): 784 -> 100 sigmoid
-> 10, softmax cross-entropy, plain SGD lr 0.001, batch 100 PER WORKER (weak
scaling: global batch = 100 * N), W ~ N(0, 1), f32 compute (the reference's
dtype).  Data: synthetic MNIST-shaped batches resident in HBM.  Every timed
step does the full work: forward, loss, backward, all-reduce of the 318 KB
gradient (N > 1) and the SGD apply.

Prints ONE JSON line on rank 0; value = total samples/sec over all N GPUs.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from distributedtensorflowexample_amd.data.synthetic import mnist_like_device  # noqa: E402
from distributedtensorflowexample_amd.models.mlp import init_params  # noqa: E402
from distributedtensorflowexample_amd.train.fused_mlp import FusedMLPTrainer  # noqa: E402

METRIC = "samples/sec (whole node) MNIST MLP sync-SGD at 1/2/4/8 MI355X; scaling efficiency"


# Rehearsal mode for the multi-rank paths on a ONE-GPU box: every rank shares device 0 and
# an xGMI-IPC communicator (LL push protocol) stands in for RCCL, which refuses two ranks on
# one GPU.  Never set for real runs; the JSON records it.
SHARED_GPU = os.environ.get("DTFX_SHARED_GPU") == "1"


def _comm_label(a):
    return a.comm + ("+shared-gpu-rehearsal" if SHARED_GPU else "")


def mlp_numel():
    from distributedtensorflowexample_amd.ops import mlp_step

    return mlp_step.NPARAM


def _native_comm(world, rank, dev, max_numel):
    if SHARED_GPU:
        from distributedtensorflowexample_amd.parallel.xgmi import XgmiComm

        # LL push words take 8 B per element per peer slot: model-sized buckets (BERT's 110M
        # parameters: 3.5 GB per rank) use the flag protocol's f32 slots instead (an IPC
        # mapping of that size did not open within minutes on the shared GPU)
        small = world <= 8 and max_numel <= (4 << 20)
        return XgmiComm(rank, world, max_numel, device=dev, key="dtfx/shared",
                        protocol="push" if small else "flag",
                        timeout_s=120.0)  # peers time-share the GPU (and start skewed)
    from distributedtensorflowexample_amd.parallel.comm import NativeComm

    return NativeComm.from_process_group()


def _timing_barrier(comm, local):
    """Barrier that brackets the timed region (both sides, after torch.cuda.synchronize()).

    A gloo barrier is a TCP round trip through rank 0 (~0.1-0.3 ms), as long as a whole
    short MLP run; the ranks' GPUs already share a RCCL communicator, so the bracket is a
    one-element RCCL all-reduce + synchronize (a device-side rendezvous of every rank).
    Falls back to the process-group barrier where there is no RCCL communicator (the
    shared-GPU rehearsal, --comm torch)."""
    from distributedtensorflowexample_amd.parallel.comm import NativeComm

    if isinstance(comm, NativeComm):
        one = torch.zeros(1, device=comm.device)

        def bar():
            comm.allreduce_sum_(one)
            torch.cuda.synchronize()

        bar()  # first call of this size: RCCL sets up outside the timed region
        return bar
    if dist.get_backend() == "nccl":
        return lambda: dist.barrier(device_ids=[local])
    return dist.barrier


def _large_bucket_comm(a, comm, world, rank, dev, max_numel):
    """BERT / ResNet gradient buckets: RCCL, or (``--comm auto``, N > 1) RCCL with the buckets
    where the xGMI bandwidth-mode two-shot measured faster routed to it
    (parallel/select.py::pick_large_allreduce, probe recorded in the JSON)."""
    a.comm_probe = None
    if world < 2 or world > 8 or SHARED_GPU or a.comm != "auto" or comm is None:
        return comm
    from distributedtensorflowexample_amd.parallel.select import HybridComm, pick_large_allreduce

    c, a.comm_probe = pick_large_allreduce(comm, world, rank, dev, max_numel)
    a.comm = "rccl+xgmi-bw" if isinstance(c, HybridComm) else "native"
    return c


def main():
    if os.environ.get("DTFX_WATCHDOG_S"):  # debugging aid: dump every thread's stack, then exit
        import faulthandler

        faulthandler.dump_traceback_later(float(os.environ["DTFX_WATCHDOG_S"]), exit=True)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--model", choices=["mlp", "bert", "resnet50"], default="mlp",
                    help="mlp: the headline MNIST MLP (BASELINE.json metric); bert: north-star "
                         "BERT-base MLM config")
    ap.add_argument("--steps", type=int, default=None, help="default 20000 (mlp) / 30 (bert)")
    ap.add_argument("--warmup", type=int, default=None, help="default 2000 (mlp) / 5 (bert)")
    ap.add_argument("--bert_batch", type=int, default=128, help="BERT sequences per GPU")
    ap.add_argument("--seq_len", type=int, default=128)
    ap.add_argument("--bert_config", choices=["base", "tiny"], default="base")
    ap.add_argument("--resnet_batch", type=int, default=256, help="ResNet-50 images per GPU")
    ap.add_argument("--image_size", type=int, default=224)
    ap.add_argument("--batch_size", type=int, default=100)
    ap.add_argument("--learning_rate", type=float, default=0.001)
    ap.add_argument("--max_graph_steps", type=int, default=1024,
                    help="max steps per hipGraph (graphs are epoch-aligned)")
    ap.add_argument("--no_graph", action="store_true")
    ap.add_argument("--launch", choices=["auto", "graph", "host", "persistent"], default="auto",
                    help="MLP, 1 GPU: how the timed steps are issued -- graph = hipGraph "
                         "replays, host = the C++ host loop launching both kernels of every "
                         "step (no graph-submission latency), persistent = ALL K steps in one "
                         "launch of the persistent kernel (workgroups hand data to each other "
                         "as epoch-tagged granules; measured slower, explicit only), auto = "
                         "time graph / host on min(K, 2000) steps before the timed region and "
                         "use the faster")
    ap.add_argument("--comm", choices=["auto", "native", "xgmi", "torch"], default="auto",
                    help="native: the framework's C++ RCCL communicator (gloo control plane); "
                         "xgmi: one-shot peer-memory all-reduce over xGMI (small buckets); "
                         "auto (MLP, N>1): verify xgmi against RCCL, time both, use the faster; "
                         "torch: torch.distributed nccl(=RCCL) process group")
    ap.add_argument("--engine",
                    choices=["auto", "fused", "fused2", "fused2x", "factor", "factor2",
                             "allreduce"],
                    default="auto",
                    help="MLP, N>1: fused = gradient exchange inside the backward kernel (xGMI LL "
                         "push); factor = sufficient-factor exchange (dz1 all-gathered in the "
                         "head kernel, global W1 gradient formed on every rank from every "
                         "rank's resident batch); fused2 / factor2 = the same exchanges in the "
                         "two-launch pipelined step; allreduce = separate all-reduce launch; "
                         "auto = verify + time all, keep the fastest")
    ap.add_argument("--dataset_size", type=int, default=55000)
    ap.add_argument("--dp", action="store_true",
                    help="use the data-parallel path (gradient all-reduce) even on 1 GPU")
    a = ap.parse_args()
    if os.environ.get("DTFX_STACKS_ON_USR1") == "1":  # (diagnostics: all threads' stacks)
        import faulthandler
        import signal

        faulthandler.register(signal.SIGUSR1, all_threads=True)
    if a.steps is None:
        a.steps = {"mlp": 20000, "bert": 30, "resnet50": 20}[a.model]
    if a.warmup is None:
        a.warmup = 2000 if a.model == "mlp" else 5

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("DTFX_BENCH_PIN") == "1":
        # A/B knob: this rank's host thread (and the HIP runtime threads it starts) on one CPU
        # of its GPU's NUMA node, chosen before the GPU is touched -- the MLP's short timed
        # region issues ~40 launches from the host, so scheduler migrations show in it
        from distributedtensorflowexample_amd.config import first_gpu_numa_node_sysfs, pin_to_numa_node

        node = first_gpu_numa_node_sysfs(index=local)
        pin_to_numa_node(0 if node is None else node, 1, 2 + 2 * local)
    from distributedtensorflowexample_amd.config import apply_hip_schedule

    apply_hip_schedule()  # DTFX_HIP_SCHED (unset: the runtime's default wait)
    if a.comm == "auto" and world == 1:
        a.comm = "native"
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            sys.exit("--gpus %d needs torch.distributed.run with %d processes" % (a.gpus, a.gpus))
    if SHARED_GPU:
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if a.comm == "torch":
            dist.init_process_group("nccl", device_id=dev)
        else:  # control plane over TCP/gloo; gradients over the native RCCL / xGMI communicator
            import datetime

            # a collective that cannot complete errors out in minutes instead of hanging
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=600))

    if a.model == "bert":
        return bench_bert(a, world, rank, local, dev)
    if a.model == "resnet50":
        return bench_resnet(a, world, rank, local, dev)

    # identical replicas: the counter-based Philox init gives every rank the
    # same parameters from the same seed (no broadcast needed; verified below)
    params = init_params(dev, seed=1234)
    x, y = mnist_like_device(a.dataset_size, seed=100 + rank, device=dev)
    x_all = None
    if 2 <= world <= 8 and a.engine in ("auto", "factor", "factor2") and a.comm != "torch":
        # every rank's batch stream resident on every GPU (each reference process loads the
        # whole dataset, main.py:43-44): the factor engine then exchanges only dz1
        x_all = torch.empty(world, a.dataset_size, 784, device=dev)
        for q in range(world):
            x_all[q].copy_(x if q == rank else mnist_like_device(a.dataset_size, seed=100 + q,
                                                                 device=dev)[0])
        x = x_all[rank]

    allreduce = fused_comm = factor_comm = None
    if world > 1:
        from distributedtensorflowexample_amd.parallel.comm import TorchComm

        if a.comm == "torch":
            comm = TorchComm()
        else:
            comm = _native_comm(world, rank, dev, mlp_numel())
        rendezvous = comm  # RCCL communicator kept for the timing barrier
        # shared-GPU rehearsal: the peers time-share one device, so an xGMI wait lasts longer
        tmo = 60.0 if SHARED_GPU else 2.0
        if a.comm != "torch":
            if a.comm in ("xgmi", "auto"):
                from distributedtensorflowexample_amd.parallel.select import pick_small_allreduce
                from distributedtensorflowexample_amd.parallel.xgmi import XgmiComm

                comm, probe = pick_small_allreduce(comm, a.comm, world, rank, dev, timeout_s=tmo)
                a.comm_probe = probe
                a.comm = ("xgmi-" + comm.protocol) if isinstance(comm, XgmiComm) else "native"
            if a.engine != "allreduce":
                # exchange fused into the backward kernel vs separate all-reduce: measured
                from distributedtensorflowexample_amd.parallel.select import pick_mlp_engine

                kind, c, eprobe = pick_mlp_engine(params, x, y, a.batch_size, a.learning_rate,
                                                  comm, world, rank, dev, mode=a.engine,
                                                  x_all=x_all, timeout_s=tmo)
                a.engine_probe = eprobe
                if kind in ("fused", "fused2", "fused2x"):
                    fused_comm, a.comm = c, "xgmi-fused-push"
                elif kind in ("factor", "factor2"):
                    factor_comm, a.comm = c, "xgmi-factor-allgather"
                a.engine_pipeline = kind in ("fused2", "fused2x", "factor2")
                a.engine_kind = kind
        if factor_comm is None:
            x_all = None
        allreduce = None if (fused_comm is not None or factor_comm is not None) else comm.allreduce_sum_
        chk = params.double().sum().reshape(1).cpu()
        ref = chk.clone()
        if a.comm == "torch":  # nccl process group: device tensors
            ref = ref.to(dev)
        dist.broadcast(ref, 0)  # else the gloo control plane
        if not torch.equal(chk, ref.cpu()):
            raise RuntimeError("replicas are not identical after init")

    if world == 1 and a.dp:  # 1-rank communicator: exercises the sync-DP path on one GPU
        if a.comm == "xgmi":
            from distributedtensorflowexample_amd.ops import mlp_step
            from distributedtensorflowexample_amd.parallel.xgmi import XgmiComm

            comm = XgmiComm(0, 1, mlp_step.NPARAM, device=dev, store=dist.HashStore())
        else:
            from distributedtensorflowexample_amd.parallel.comm import NativeComm

            comm = NativeComm(0, 1, store=dist.HashStore())
        allreduce = comm.allreduce_sum_
    tr = FusedMLPTrainer(params, x, y, batch_size=a.batch_size, learning_rate=a.learning_rate,
                         allreduce=allreduce, world_size=world,
                         max_graph_steps=a.max_graph_steps, fused_comm=fused_comm,
                         factor_comm=factor_comm, x_all=x_all, rank=rank,
                         pipeline=getattr(a, "engine_pipeline", True))
    barrier = _timing_barrier(rendezvous, local) if world > 1 else None
    use_graph = not a.no_graph

    tr.run(a.warmup, use_graph)
    # How the timed steps are issued.  A graph replay pays a fixed submission latency
    # (t(n) = 17 us + 8.2 us * n, tools/probes/graph_fixed_cost.py) that a short timed region
    # (the driver's K = 20) feels; the C++ host loop (FusedMLPTrainer.run_launched) launches
    # the first kernel at once but pays a host launch per kernel.  In a fresh process the
    # host loop's first launches were slow (10.6-14.9 us/step at K = 20 against 10.0 for the
    # graph), so for K <= 200 both are warmed and timed here on K steps (untimed; the JSON
    # records every step run before the clock as pre_timing_steps) and the faster is used.
    # Longer regions take the graph: its fixed cost is amortised, while the host loop falls
    # behind once the launch queue fills (K = 20000: 9.02 us/step against 8.15 for the graph,
    # though both timed 8.3-8.4 on a 200-step probe).
    launch = "graph" if use_graph else "eager"
    a.launch_probe = None
    if a.launch == "persistent" and not tr.persistent_ok:
        sys.exit("--launch persistent: single GPU, batch <= 128 only")
    # The persistent engine (--launch persistent) is not an auto candidate: it measured
    # 9.0-9.2 us/step against the graph's 8.2 on every box (profiles/r2/persistent/), so
    # probing it would only lengthen the startup.
    cands = []
    if use_graph and tr.host_loop_ok and a.launch == "auto":
        cands = ["graph"] + (["host"] if a.steps <= 200 else [])
    if a.launch == "host" and tr.host_loop_ok:
        launch = "host"
    if a.launch == "persistent":
        launch = "persistent"
    if launch in ("host", "persistent") or len(cands) > 1:
        kp = min(a.steps, 2000)

        def run_k(mode):
            if mode == "host":
                tr.run_launched(kp, flush=True)  # (the flush launched by the same call)
            elif mode == "persistent":
                tr.run_persistent(kp)
            else:
                tr.run(kp)
            tr.flush()

        probe = {m: [] for m in cands}
        if tr.host_loop_ok:
            tr.run_launched(max(a.warmup, 8))  # warm the direct-launch path
        if tr.persistent_ok and (launch == "persistent" or "persistent" in cands):
            tr.run_persistent(max(a.warmup, 8))  # first launch: granule buffer + code object
            tr.check()
            tr.run(1, use_graph=False)
        for _ in range(3 if cands else 0):
            for mode in probe:
                if mode == "graph":
                    tr.prepare(kp)
                torch.cuda.synchronize()
                t_0 = time.perf_counter()
                run_k(mode)
                torch.cuda.synchronize()
                probe[mode].append((time.perf_counter() - t_0) * 1e6 / kp)
                tr.run(1, use_graph=False)  # pending update again, as after the warmup
        if cands:
            tr.check()
            med = {m: sorted(v)[len(v) // 2] for m, v in probe.items()}
            if world > 1:  # the same choice on every rank: max over ranks of each median
                names = sorted(med)
                t = torch.tensor([med[m] for m in names], dtype=torch.float64)
                t = t if a.comm != "torch" else t.to(dev)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                med = dict(zip(names, t.cpu().tolist()))
            launch = min(med, key=lambda m: (med[m], m))
            a.launch_probe = {m: round(v, 3) for m, v in med.items()}
    if launch == "graph":
        tr.prepare(a.steps)
    if launch == "persistent":
        tr.flush()  # the warmup's pending update lands before the clock (it is not a timed step)
    pre_steps = tr.global_step()
    if barrier:
        barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if launch == "host":
        tr.run_launched(a.steps, flush=True)  # the last step's update: one more launch, same call
    elif launch == "persistent":
        tr.run_persistent(a.steps)  # every update applied inside the launch
    else:
        tr.run(a.steps, use_graph)
    if launch != "persistent":  # (the persistent launch leaves nothing pending)
        tr.flush()  # the last step's deferred update is part of the timed work
    torch.cuda.synchronize()
    if barrier:
        barrier()
    elapsed = time.perf_counter() - t0
    tr.check()  # raises if a persistent-engine hand-off ever timed out
    for c in ((comm, fused_comm, factor_comm) if world > 1 else ()):
        if hasattr(c, "check"):
            c.check()  # raises if an xGMI exchange ever timed out

    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        t = t if a.comm != "torch" else t.to(dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    loss, acc = tr.stats()
    identical = None
    if world > 1:  # after the clock: the sync replicas must still be bit-identical
        chk = tr.params.double().sum().reshape(1).cpu()
        ref = chk.clone()
        ref = ref if a.comm != "torch" else ref.to(dev)
        dist.broadcast(ref, 0)
        same = torch.tensor([1 if torch.equal(chk, ref.cpu()) else 0], dtype=torch.int32)
        same = same if a.comm != "torch" else same.to(dev)
        dist.all_reduce(same, op=dist.ReduceOp.MIN)
        identical = bool(same.item())
    ms = elapsed * 1e3 / a.steps
    value = a.batch_size * world * a.steps / elapsed
    if rank == 0:
        print(json.dumps({
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "samples/sec",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 6),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (MNIST-shaped, device-resident), random-init N(0,1) weights",
            "config": {
                "model": "MNIST MLP 784-100(sigmoid)-10, softmax-xent, SGD lr=%g" % a.learning_rate,
                "global_batch": a.batch_size * world,
                "per_gpu_batch": a.batch_size,
                "seq_len": None,
                "parallelism": "dp%d" % world,
                "comm": _comm_label(a) if (world > 1 or a.dp) else "none",
                "hipgraph": launch == "graph",
                "launch": launch,
                "engine": getattr(a, "engine_kind", "allreduce" if allreduce else "single"),
                "launches_per_step": (round(1.0 / a.steps, 6) if launch == "persistent"
                                      else 2 if tr.pipelined else 3),
            },
            "comm_probe_us": getattr(a, "comm_probe", None),
            "engine_probe_us_per_step": getattr(a, "engine_probe", None),
            "launch_probe_us_per_step": a.launch_probe,
            "pre_timing_steps": pre_steps,
            "final_loss": round(loss, 5),
            "final_train_acc": round(acc, 4),
            "global_step": tr.global_step(),
            "replicas_identical": identical,
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_bert(a, world, rank, local, dev):
    """North-star config: BERT-base MLM pre-training step, bf16, sync DP over RCCL."""
    from distributedtensorflowexample_amd.models.bert import BertConfig
    from distributedtensorflowexample_amd.train.bert_trainer import BertTrainer

    comm = None
    if world > 1:
        from distributedtensorflowexample_amd.parallel.comm import TorchComm

        comm = _native_comm(world, rank, dev, 160 << 20) if a.comm != "torch" else TorchComm()
    cfg = BertConfig.base() if a.bert_config == "base" else BertConfig.tiny()
    rendezvous, comm = comm, _large_bucket_comm(a, comm, world, rank, dev, 24 << 20)
    tr = BertTrainer(cfg, a.bert_batch, a.seq_len, dev, comm=comm, data_seed=17 + rank)
    use_graph = not a.no_graph
    tr.run(a.warmup, use_graph)
    barrier = _timing_barrier(rendezvous, local) if world > 1 else None
    if barrier:
        barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.run(a.steps, use_graph)
    torch.cuda.synchronize()
    if barrier:
        barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        t = t if a.comm != "torch" else t.to(dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    loss, acc = tr.stats()
    ms = elapsed * 1e3 / a.steps
    seqs = a.bert_batch * world * a.steps / elapsed
    if rank == 0:
        print(json.dumps({
            "metric": "sequences/sec (whole node) BERT-%s MLM pre-training, seq %d" % (a.bert_config,
                                                                                     a.seq_len),
            "value": round(seqs, 1), "unit": "sequences/sec", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic MLM (Markov-chain token ids, 15% masked: 80% [MASK] / 10% "
                    "random / 10% kept; 8 device-resident batches rotated), random-init weights",
            "config": {"model": "BERT-%s MLM (L%d H%d A%d, vocab %d)" % (
                a.bert_config, cfg.layers, cfg.hidden, cfg.heads, cfg.vocab_size),
                "global_batch": a.bert_batch * world, "per_gpu_batch": a.bert_batch,
                "seq_len": a.seq_len, "parallelism": "dp%d" % world,
                "comm": _comm_label(a) if world > 1 else "none", "hipgraph": use_graph,
                "optimizer": "AdamW (fused, f32 master)"},
            "model_tflops_per_gpu": round(tr.flops_per_step() / (ms * 1e-3) / 1e12, 1),
            "comm_probe_us": getattr(a, "comm_probe", None),
            "final_loss": round(loss, 4), "final_mlm_acc": round(acc, 4),
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_resnet(a, world, rank, local, dev):
    """North-star config: ResNet-50 synthetic ImageNet, bf16, sync DP over RCCL."""
    from distributedtensorflowexample_amd.train.resnet_trainer import ResNetTrainer

    comm = None
    if world > 1:
        from distributedtensorflowexample_amd.parallel.comm import TorchComm

        comm = _native_comm(world, rank, dev, 32 << 20) if a.comm != "torch" else TorchComm()
    rendezvous, comm = comm, _large_bucket_comm(a, comm, world, rank, dev, 8 << 20)
    tr = ResNetTrainer(a.resnet_batch, dev, comm=comm, image_size=a.image_size, data_seed=rank)
    use_graph = not a.no_graph
    tr.run(a.warmup, use_graph)
    barrier = _timing_barrier(rendezvous, local) if world > 1 else None
    if barrier:
        barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.run(a.steps, use_graph)
    torch.cuda.synchronize()
    if barrier:
        barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        t = t if a.comm != "torch" else t.to(dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    loss, acc = tr.stats()
    ms = elapsed * 1e3 / a.steps
    if rank == 0:
        print(json.dumps({
            "metric": "images/sec (whole node) ResNet-50 v1.5 training, synthetic ImageNet",
            "value": round(a.resnet_batch * world * a.steps / elapsed, 1), "unit": "images/sec",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (random %dx%d images, device-resident), random-init weights"
                    % (a.image_size, a.image_size),
            "config": {"model": "ResNet-50 v1.5 (BN train mode, momentum SGD)",
                       "global_batch": a.resnet_batch * world, "per_gpu_batch": a.resnet_batch,
                       "seq_len": None, "parallelism": "dp%d" % world,
                       "comm": _comm_label(a) if world > 1 else "none", "hipgraph": use_graph},
            "comm_probe_us": getattr(a, "comm_probe", None),
            "final_loss": round(loss, 4), "final_train_acc": round(acc, 4),
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
