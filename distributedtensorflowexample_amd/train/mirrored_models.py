"""``main.py --strategy mirrored --model {bert,resnet50}``: the north-star models under
the same CLI, observability and fault-tolerance contract as the reference's MLP.

* one process per GPU (``torch.distributed.run``; gloo control plane, RCCL data);
* the chief's :class:`~..train.supervisor.Supervisor` restores the latest TF-V2
  checkpoint from ``--logdir`` (or initialises) and saves every
  ``--save_model_secs`` (variables in the TF layout of ``models.bert.tf_variables``
  / ``models.resnet.tf_variables`` + ``global_step``); the other ranks receive the
  chief's parameters by broadcast, so a killed job resumes where its last checkpoint
  left off (``tests/test_fault_resume.py``);
* ``step: N | cost: C | speed: S step/sec`` every ``--log_every`` steps (worker.py:145-146),
  TensorBoard loss/accuracy scalars into ``<logdir>_<rank>``.

The reference has no such models (it trains an MLP, worker.py:47-79); the
contract mirrors worker.py:98-159.
"""
from __future__ import annotations

import os
import time

import torch
import torch.distributed as dist

from ..parallel.comm import NativeComm, TorchComm
from ..parallel.watchdog import init_process_group_with_timeout, maybe_inject_fault, watch_peers
from ..parallel.select import check_comm_collective
from ..utils.summary import FileWriter
from .saver import FastSaver
from .supervisor import Supervisor


def _dist_env():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def train_model_mirrored(flags, log=print):
    rank, world, local = _dist_env()
    use_gpu = torch.cuda.is_available() and flags.device != "cpu"
    if world > 1 and not dist.is_initialized():
        init_process_group_with_timeout(  # control plane; tensors over RCCL on GPU
            "gloo", getattr(flags, "dist_timeout_secs", None))
    if use_gpu:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        comm = NativeComm.from_process_group() if world > 1 else None
        if comm is not None and 2 <= world <= 8 and os.environ.get("DTFX_COMM_LARGE", "auto") == "auto":
            # large gradient buckets: RCCL, or the xGMI bandwidth-mode two-shot from the bucket
            # size where it measured faster (the same decision on every rank)
            from ..parallel.select import pick_large_allreduce

            comm, _ = pick_large_allreduce(
                comm, world, rank, dev, (24 << 20) if flags.model == "bert" else (8 << 20),
                peer_timeout_s=float(getattr(flags, "peer_timeout_secs", 60.0) or 0.0))
    else:
        dev = torch.device("cpu")
        comm = TorchComm() if world > 1 else None
    is_chief = rank == 0
    if getattr(flags, "zero1", False) and world > 1 and flags.model != "bert":
        raise ValueError("--zero1 is not implemented for --model %s (replicated fused "
                         "optimizer); it applies to bert and the autograd MLP path" % flags.model)
    tiny = flags.model_config == "tiny"
    if flags.model == "bert":
        from ..models import bert as M
        from .bert_trainer import BertTrainer

        cfg = M.BertConfig.tiny() if tiny else M.BertConfig.base()
        # the owner-sharded AdamW is the world > 1 default (--zero1 keeps it on explicitly;
        # DTFX_BERT_ZERO1=0 turns it off)
        tr = BertTrainer(cfg, flags.batch_size, flags.seq_len, dev, comm=comm,
                         lr=flags.learning_rate, seed=flags.seed, data_seed=17 + rank,
                         zero1=True if getattr(flags, "zero1", False) else None)
    elif flags.model == "resnet50":
        from ..models import resnet as M
        from .resnet_trainer import ResNetTrainer

        stages = [(8, 1, 1), (16, 1, 2)] if tiny else M.STAGES
        ncls = 10 if tiny else 1000
        tr = ResNetTrainer(flags.batch_size, dev, comm=comm, lr=flags.learning_rate,
                           seed=flags.seed, image_size=32 if tiny else flags.image_size,
                           stages=stages, num_classes=ncls, data_seed=rank)
    else:
        raise ValueError("--model must be bert or resnet50 here (mlp: train_mirrored)")
    model = tr.model
    state = {"step": 0}

    def global_step():
        return state["step"]

    def save_vars():
        v = M.tf_variables(model)
        v["global_step"] = torch.tensor(global_step(), dtype=torch.int64)
        return v

    def restore(values):
        M.load_tf_variables(model, values)
        state["step"] = int(values["global_step"])

    saver = FastSaver(assign=restore)
    writer = FileWriter("%s_%d" % (flags.logdir, rank)) if flags.logdir else None
    sv = Supervisor(is_chief=is_chief, logdir=flags.logdir if is_chief else None,
                    saver=saver if is_chief else None, summary_writer=writer,
                    global_step=global_step, save_model_secs=flags.save_model_secs,
                    save_summaries_secs=flags.save_summaries_secs, save_variables=save_vars,
                    checkpoint_on_main_thread=True)  # never read parameters mid-step
    steps_total = int(flags.training_steps)
    # fail-fast: a rank whose peer died aborts its communicator and exits (non-zero)
    with watch_peers(comm, float(getattr(flags, "peer_timeout_secs", 60.0) or 0.0)), \
            sv.managed_session():
        if is_chief and sv.restored_from is not None:
            log("Restored %s (global_step %d)" % (sv.restored_from, global_step()))
        if world > 1:  # every replica starts from the chief's parameters and step
            p = model.params.master
            comm.broadcast_(p, 0)
            from ..ops import transformer as TR

            TR.cast_bf16(p, model.params.bf)
            s = torch.tensor([global_step()], dtype=torch.int64)
            dist.broadcast(s, 0)
            state["step"] = int(s.item())
        use_graph = use_gpu
        t0, s0 = time.time(), global_step()
        while not sv.should_stop() and global_step() < steps_total:
            tr.step(use_graph)
            state["step"] += 1
            step = global_step()
            maybe_inject_fault(rank, step)
            k = int(getattr(flags, "check_replicas_every", 0) or 0)
            logstep = step % int(flags.log_every) == 0 or step == steps_total
            # owner-sharded optimizer: the other ranks' shards of the last update arrive with
            # the next step's gathers; complete them (a collective: the same steps on every
            # rank) wherever parameters are read -- replica checks and the chief's checkpoints,
            # which then happen only at these steps
            sharded = getattr(tr, "zero1", False)
            synced = False
            if sharded and (logstep or (k > 0 and step % k == 0)):
                tr.sync_params()
                synced = True
            if k > 0 and world > 1 and step % k == 0:
                from ..parallel.mirrored import assert_replicas_identical

                assert_replicas_identical(comm, model.params.master, world, step)
            if world > 1 and use_gpu:
                # a timed-out xGMI bucket all-reduce leaves diverged replicas: stop on every
                # rank at the next log step (same step everywhere: a collective check), and
                # never let the chief checkpoint parameters its own comm reports as partial
                if logstep:
                    check_comm_collective(comm, "step %d" % step)
                elif is_chief and sv.checkpoint_pending() and getattr(comm, "failed", None) \
                        and comm.failed():
                    raise RuntimeError("xGMI all-reduce timed out before a checkpoint")
            if synced or not sharded:
                sv.service()  # a requested checkpoint, between steps
            if logstep:
                loss, acc = tr.stats()
                if writer is not None:
                    writer.add_scalars({"loss": loss, "accuracy": acc}, step)
                if is_chief:
                    el = time.time() - t0
                    log("step: {}\t| cost: {}\t| speed: {}step/sec".format(
                        step, loss, float((step - s0) / max(el, 1e-9))))
                    t0, s0 = time.time(), step
        if getattr(tr, "zero1", False):
            tr.sync_params()  # (every rank) the final checkpoint reads complete parameters
        if is_chief:
            sv.save_checkpoint()
    return global_step()
