"""Sync data-parallel training loop of the reference MLP (``--strategy mirrored``).

One process per GPU (env RANK / WORLD_SIZE / LOCAL_RANK from the launcher
or torch.distributed.run).  GPU: the fused two-launch step + the native RCCL
all-reduce, hipGraph-replayed per epoch (train/fused_mlp.py).  CPU (gloo):
the autograd MnistMLP wrapped in DistributedDataParallel.

Observability mirrors the reference: ``step / cost / speed`` prints every
``log_every`` steps (speed in global steps/sec; samples/sec = speed *
batch_size * replicas), test accuracy every ``eval_every`` steps, loss and
accuracy summaries (bulk-written from the device stats ring), and chief
checkpoints in TF V2 format with the reference's variable names.
"""
from __future__ import annotations

import os
import time

import torch
import torch.distributed as dist

from ..models import mlp as mlp_model
from ..ops import mlp_step, nn, optim
from ..parallel.comm import NativeComm, TorchComm
from ..parallel.watchdog import init_process_group_with_timeout, maybe_inject_fault, watch_peers
from ..optim import GradientDescentOptimizer
from ..parallel.mirrored import DistributedDataParallel
from ..parallel.sharded import ShardedOptimizer
from ..utils.summary import FileWriter
from .fused_mlp import FusedMLPTrainer
from .saver import FastSaver
from .supervisor import Supervisor
from .worker import flat_to_tf_vars, tf_vars_to_flat


def _dist_env():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def _mlp_graph(batch, lr):
    """The reference MLP's graph for the chief's Supervisor (names from a variable registry
    built like the async worker's, utils/graph.py)."""
    from .. import variables as vs
    from ..models.dense import make_ps_model
    from ..utils.graph import reference_mlp_graph
    from .worker import build_worker_variables

    gv, tv = build_worker_variables(make_ps_model("mlp", "", None), vs.VariableRegistry())
    return reference_mlp_graph(gv, tv, 0, batch_size=batch, learning_rate=lr)


def train_mirrored(flags, dataset, log=print, max_steps=None):
    rank, world, local = _dist_env()
    use_gpu = torch.cuda.is_available() and flags.device != "cpu"
    if world > 1 and not dist.is_initialized():
        init_process_group_with_timeout(  # control plane; tensors over RCCL on GPU
            "gloo", getattr(flags, "dist_timeout_secs", None))
    shared_gpu = os.environ.get("DTFX_SHARED_GPU") == "1"
    if use_gpu:
        # DTFX_SHARED_GPU=1 (rehearsal on a one-GPU box only): every rank on device 0 and an
        # xGMI-IPC communicator in place of RCCL, which refuses two ranks on one GPU
        local = 0 if shared_gpu else local
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        comm = None
        if world > 1 and shared_gpu:
            from ..parallel.xgmi import XgmiComm

            comm = XgmiComm(rank, world, mlp_step.NPARAM, device=dev, key="dtfx/mirrored/shared",
                            protocol="push", timeout_s=120.0)
        elif world > 1:
            comm = NativeComm.from_process_group()
        if getattr(flags, "zero1", False) and world > 1:
            # the fused GPU engines exchange gradients inside their kernels; a 1/N-sharded
            # update of a 318 KB model would only add two collectives per step
            raise ValueError("--zero1 is implemented on the autograd (CPU) mirrored path; the "
                             "fused GPU MLP engines replicate the update")
        if (comm is not None and not shared_gpu
                and os.environ.get("DTFX_MLP_COMM", "auto") != "rccl"):
            # the 318 KB gradient is latency bound: xGMI one-shot when verified and faster
            from ..parallel.select import pick_small_allreduce

            comm, _ = pick_small_allreduce(comm, "auto", world, rank, dev)
    else:
        dev = torch.device("cpu")
        comm = TorchComm() if world > 1 else None
    is_chief = rank == 0
    steps_total = int(flags.training_steps if max_steps is None else max_steps)
    B = int(flags.batch_size)

    params = mlp_model.init_params(dev, seed=int(flags.seed))  # identical on every rank
    # each replica trains on its own shard of the (shuffled) training set
    tr_x = torch.from_numpy(dataset.train.images[rank::world]).float()
    tr_y = torch.from_numpy(dataset.train.labels[rank::world])
    tr_y = (tr_y.argmax(1) if tr_y.ndim == 2 else tr_y).to(torch.int32)

    writer = FileWriter(flags.logdir + "_%d" % rank) if is_chief else None
    # host mirror of global_step, advanced by the training loop only: the Supervisor's
    # service threads read it instead of touching trainer/device state
    state = {"step": 0}

    if use_gpu:
        fused = factor = x_all = None
        pipe = True
        if comm is not None and os.environ.get("DTFX_MLP_COMM", "auto") != "rccl":
            # exchange engine (fused into the backward kernel / factor all-gather) when
            # verified and faster than the all-reduce engine
            from ..parallel.select import pick_mlp_engine

            if world <= 8:
                # every process holds the whole training set (like every reference
                # process, main.py:43-44): equal-length shards of all ranks, resident
                n = min(len(dataset.train.images[q::world]) for q in range(world))
                x_all = torch.stack([torch.from_numpy(dataset.train.images[q::world][:n]).float()
                                     for q in range(world)]).to(dev).contiguous()
                tr_x, tr_y = x_all[rank], tr_y[:n]
            kind, c, _ = pick_mlp_engine(params, tr_x.to(dev), tr_y.to(dev), B,
                                         flags.learning_rate, comm, world, rank, dev, x_all=x_all,
                                         mode=os.environ.get("DTFX_MLP_ENGINE", "auto"))
            fused = c if kind in ("fused", "fused2", "fused2x") else None
            factor = c if kind in ("factor", "factor2") else None
            pipe = kind not in ("fused", "factor")  # fused2 / factor2: two-launch variants
        tr = FusedMLPTrainer(params, tr_x, tr_y, B, flags.learning_rate,
                             allreduce=comm.allreduce_sum_ if (comm and not (fused or factor))
                             else None, world_size=world, fused_comm=fused, factor_comm=factor,
                             x_all=x_all if factor is not None else None, rank=rank,
                             pipeline=pipe if comm is not None else True)
        # tr.snapshot() never starts a peer exchange on ONE rank and never changes the
        # replicas' update sequence (the all-reduce engine's pending gradient is applied to a
        # copy); the pipelined exchange engines have nothing pending at the checkpoint /
        # eval / replica-check points, because the loop below reads each chunk's stats on
        # EVERY rank (stats_range flushes there, collectively)
        get_params = tr.snapshot
        step_fn = None
    else:
        model = mlp_model.MnistMLP(flat=params)
        zero1 = bool(getattr(flags, "zero1", False)) and comm is not None
        ddp = DistributedDataParallel(model, comm, shard=zero1) if comm else None
        zopt = (ShardedOptimizer(GradientDescentOptimizer(flags.learning_rate), ddp)
                if zero1 else None)
        state["pos"] = 0
        get_params = lambda: model.flat.detach().clone()  # noqa: E731

        def step_fn():
            i = state["pos"]
            n = tr_x.shape[0] // B
            xb, yb = tr_x[(i % n) * B:(i % n + 1) * B], tr_y[(i % n) * B:(i % n + 1) * B]
            state["pos"] = i + 1
            if ddp:
                ddp.reset()
            else:
                model.flat.grad = None
            loss, acc = model.loss(xb, yb)
            loss.backward()
            if zopt is not None:  # reduce-scatter -> owner SGD on 1/world -> all-gather
                zopt.step()
                return float(loss), float(acc)
            if ddp:
                ddp.finish()
                g = ddp.flat_grad[:model.flat.numel()]
            else:
                g = model.flat.grad
            with torch.no_grad():
                optim.sgd_(model.flat.data, g, flags.learning_rate)
            return float(loss), float(acc)

    saver = FastSaver({n: None for n in
                       ("global/dense/kernel", "global/dense/bias", "global/dense_1/kernel",
                        "global/dense_1/bias", "global/global_step")})

    def save_vars():
        v = {k: t.contiguous() for k, t in flat_to_tf_vars(get_params().cpu()).items()}
        v["global/global_step"] = torch.tensor(global_step(), dtype=torch.int32)
        return v

    def global_step():
        return tr.global_step() if use_gpu else state.get("pos", 0)

    def published_step():
        return state["step"]

    def restore(values):
        p = torch.zeros(mlp_step.NPARAM)
        tf_vars_to_flat(values, p)
        if use_gpu:
            tr.load_params(p.to(dev))
            tr.ws.set_global_step(int(values["global/global_step"]))
            tr.pos = int(values["global/global_step"]) % tr.nbatches
        else:
            model.flat.data.copy_(p)
            state["pos"] = int(values["global/global_step"])
        state["step"] = int(values["global/global_step"])

    saver.assign = restore
    # checkpoints are taken by the training loop between chunks (Supervisor.service): the
    # fused trainer's deferred update may only be flushed where every rank flushes it
    sv = Supervisor(is_chief=is_chief, logdir=flags.logdir if is_chief else None,
                    saver=saver if is_chief else None, summary_writer=writer,
                    global_step=published_step, save_model_secs=flags.save_model_secs,
                    save_summaries_secs=flags.save_summaries_secs, save_variables=save_vars,
                    checkpoint_on_main_thread=True, graph=_mlp_graph(B, flags.learning_rate))

    test_x = torch.from_numpy(dataset.test.images).float().to(dev)
    test_y = dataset.test.labels.argmax(1) if dataset.test.labels.ndim == 2 else dataset.test.labels

    def test_accuracy():
        p = get_params()
        W1t, b1, W2t, b2 = mlp_step.unflatten(p)
        h = nn.gemm(test_x, W1t, trans_b=True, bias=b1, act="sigmoid")
        logits = nn.gemm(h, W2t, trans_b=True, bias=b2)
        return float((logits.argmax(1).cpu().numpy() == test_y).mean())

    history = []
    # fail-fast: a rank whose peer died aborts its communicator and exits (non-zero)
    with watch_peers(comm, float(getattr(flags, "peer_timeout_secs", 60.0) or 0.0)), \
            sv.managed_session():
        if world > 1 and sv.restored_from is not None:
            pass  # chief-only restore: other ranks broadcast below
        if world > 1:  # replicas start identical (restored or initialised on the chief)
            p = get_params()
            if comm is not None:
                comm.broadcast_(p, 0)
            # ... at the chief's global step (a restored chief resumes mid-run; the other
            # ranks must run exactly as many steps, or they wait in a collective forever)
            s = torch.tensor([global_step()], dtype=torch.int64)
            dist.broadcast(s, 0)
            s = int(s.item())
            if use_gpu:
                tr.load_params(p)
                tr.ws.set_global_step(s)
                tr.pos = s % tr.nbatches
            else:
                model.flat.data.copy_(p)
                state["pos"] = s
        chunk = int(flags.log_every)
        state["step"] = global_step()
        start_time, start_step = time.time(), state["step"]
        while not sv.should_stop():
            s0 = global_step()
            n = min(chunk - (s0 % chunk) if s0 % chunk else chunk, steps_total - s0)
            if n <= 0:
                break
            if use_gpu:
                tr.run(n)
                stats = tr.stats_range(s0, s0 + n)
            else:
                stats = torch.tensor([step_fn() for _ in range(n)])
            step = global_step()
            state["step"] = step
            maybe_inject_fault(rank, step)
            if writer is not None:
                writer.add_scalar_series(["loss", "accuracy"], range(s0, s0 + n), stats.tolist())
            cost = float(stats[-1, 0])
            history.append((step, cost, float(stats[-1, 1])))
            if is_chief and step % chunk == 0:
                if use_gpu:
                    torch.cuda.synchronize()
                elapsed = time.time() - start_time
                log("step: {}\t| cost: {}\t| speed: {}step/sec".format(
                    step, cost, float((step - start_step) / max(elapsed, 1e-9))))
                start_time, start_step = time.time(), step
            if is_chief and step % int(flags.eval_every) == 0:
                log("test accuracy: {}".format(test_accuracy()))
            k = int(getattr(flags, "check_replicas_every", 0) or 0)
            if k > 0 and world > 1 and step % k == 0:
                from ..parallel.mirrored import assert_replicas_identical

                assert_replicas_identical(comm, get_params(), world, step)
            sv.service()  # a requested checkpoint, on this thread, between chunks
            if step >= steps_total:
                break
        if is_chief:
            sv.save_checkpoint()
    return history, get_params()


def shutdown_mirrored():
    """Orderly end of a mirrored run (the CLI's, main.py): every rank -- the chief's final
    checkpoint included -- reaches a barrier before any process group goes away.  A rank that
    exited while the store-hosting chief was still tearing its gloo group down died in
    std::terminate at interpreter exit now and then (tests/test_cluster_e2e.py, frequent
    checkpoints)."""
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
