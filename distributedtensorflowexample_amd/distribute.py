"""``tf.distribute``-style entry points (BASELINE.json north star: "tf.train.ClusterSpec /
tf.distribute entrypoints").

The reference only uses TF 1.x between-graph replication (``replica_device_setter``,
``tf.train.Server``, worker.py:24-25, main.py:67-75); the strategies here give the same
two training modes a ``tf.distribute``-shaped front door:

* :class:`MirroredStrategy` -- synchronous data parallelism, ONE process per GPU (the
  MI355X-native layout; RCCL refuses two ranks on one GPU).  ``from_env()`` joins the
  process group from ``torchrun`` / ``TF_CONFIG``-style variables; ``run`` executes a
  replica step in this process; ``reduce`` / ``all_reduce`` / ``broadcast`` go over the
  framework's communicator (native RCCL on the GPU, gloo on the CPU);
  ``distribute_dataset`` shards a dataset by replica; ``wrap`` returns the bucketed,
  backward-overlapped :class:`~.parallel.mirrored.DistributedDataParallel`.
* :class:`MultiWorkerMirroredStrategy` -- the same over the workers of a ``TF_CONFIG``
  cluster (multi-node), rendezvous at the first task's address.
* :class:`ParameterServerStrategy` -- the reference's asynchronous PS mode: variables
  placed round-robin over the ps tasks of a :class:`~.cluster.ClusterSpec`
  (``replica_device_setter`` semantics), held by the native C++ parameter server and
  reached through :class:`~.parallel.ps.PSVariableStore`.

``scope()`` makes a strategy current for :func:`get_strategy` (tf.distribute.get_strategy).
"""
from __future__ import annotations

import contextlib
import datetime
import os

import torch
import torch.distributed as dist

from .cluster import ClusterSpec
from .parallel import mirrored as _mirrored
from .parallel.comm import TorchComm, make_comm

_CURRENT = []


class ReduceOp:
    SUM = "sum"
    MEAN = "mean"
    MAX = "max"


class _DefaultStrategy:
    """Single replica, no communication (tf.distribute's default strategy)."""

    num_replicas_in_sync = 1
    rank = 0

    def run(self, fn, args=(), kwargs=None):
        return fn(*args, **(kwargs or {}))

    def reduce(self, op, value):
        return value

    def distribute_dataset(self, *arrays):
        return arrays if len(arrays) != 1 else arrays[0]


def get_strategy():
    """The strategy of the innermost ``scope()`` (or the single-replica default)."""
    return _CURRENT[-1] if _CURRENT else _DefaultStrategy()


class _ScopeMixin:
    @contextlib.contextmanager
    def scope(self):
        _CURRENT.append(self)
        try:
            yield self
        finally:
            _CURRENT.pop()


class MirroredStrategy(_mirrored.MirroredStrategy, _ScopeMixin):
    """Synchronous all-reduce data parallelism, one process per device."""

    def __init__(self, comm=None, comm_kind="auto"):
        if comm is None:
            if not dist.is_initialized():
                raise RuntimeError("MirroredStrategy needs an initialised process group: use "
                                   "MirroredStrategy.from_env() or pass a communicator")
            comm = make_comm(comm_kind) if torch.cuda.is_available() else TorchComm()
        super().__init__(comm)

    @classmethod
    def from_env(cls, backend=None, comm_kind="auto", timeout_s=600):
        """Join the job described by RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT
        (``torch.distributed.run`` sets them) and bind LOCAL_RANK's GPU.  Control plane:
        gloo; the gradient path is the native RCCL communicator on the GPU."""
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29500")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
            if torch.cuda.is_available():
                torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
            dist.init_process_group(backend or "gloo",
                                    timeout=datetime.timedelta(seconds=timeout_s))
        return cls(comm_kind=comm_kind)

    # -- tf.distribute surface ---------------------------------------------------------
    def run(self, fn, args=(), kwargs=None):
        """Run one replica step (this process is one replica)."""
        return fn(*args, **(kwargs or {}))

    def reduce(self, op, value):
        """Cross-replica reduction of a tensor (returns a new tensor)."""
        t = value.detach().clone()
        if self.num_replicas_in_sync == 1:
            return t
        if op == ReduceOp.MAX:
            return self.comm.allreduce_max_(t)
        self.comm.allreduce_sum_(t)
        if op == ReduceOp.MEAN:
            t.div_(self.num_replicas_in_sync)
        return t

    def all_reduce_(self, t, op=ReduceOp.SUM):
        """In-place cross-replica reduction."""
        t.copy_(self.reduce(op, t))
        return t

    def distribute_dataset(self, *arrays):
        """Replica shard of each array (rows rank, rank + N, ...): every replica sees a
        disjoint slice of the data, as ``experimental_distribute_dataset`` does."""
        r, n = self.rank, self.num_replicas_in_sync
        out = tuple(a[r::n] for a in arrays)
        return out if len(out) != 1 else out[0]

    experimental_distribute_dataset = distribute_dataset

    def experimental_local_results(self, value):
        return (value,)


class MultiWorkerMirroredStrategy(MirroredStrategy):
    """``tf.distribute.experimental.MultiWorkerMirroredStrategy``: synchronous data
    parallelism over the workers (optionally a ``chief``) of a ``TF_CONFIG`` cluster,
    across nodes.  One process per GPU; the rendezvous is the TCP store on the FIRST task's
    address (chief, else worker 0), rank = position in [chief..., worker...], the local GPU
    is ``LOCAL_RANK`` (default: rank modulo the visible GPUs).  Tensors go over the
    framework's RCCL communicator (xGMI inside a node; RCCL's inter-node transport
    between them); the xGMI peer-memory paths of the MLP engines are used only where every
    rank can map every peer (selection falls back to RCCL otherwise, parallel/select.py)."""

    @classmethod
    def from_tf_config(cls, env=None, comm_kind="auto", timeout_s=600):
        cluster, task_type, task_index = ClusterSpec.from_tf_config(env)
        tasks = [("chief", a) for a in (cluster.job_tasks("chief") if "chief" in cluster.jobs
                                        else [])]
        tasks += [("worker", a) for a in cluster.job_tasks("worker")]
        if not tasks:
            raise ValueError("TF_CONFIG names no chief / worker tasks")
        ttype = task_type or "worker"
        mine = [i for i, (t, _) in enumerate(tasks) if t == ttype]
        if task_index >= len(mine):
            raise ValueError("task %s:%d is not in the cluster" % (ttype, task_index))
        rank, world = mine[task_index], len(tasks)
        if not dist.is_initialized():
            host, port = tasks[0][1].rsplit(":", 1)
            if torch.cuda.is_available():
                local = int(os.environ.get("LOCAL_RANK", rank % max(1, torch.cuda.device_count())))
                torch.cuda.set_device(local)
            dist.init_process_group("gloo", init_method="tcp://%s:%s" % (host, port), rank=rank,
                                    world_size=world,
                                    timeout=datetime.timedelta(seconds=timeout_s))
        return cls(comm_kind=comm_kind)


class ParameterServerStrategy(_ScopeMixin):
    """Asynchronous PS training over a ClusterSpec (the reference's mode).

    ``variable_store(specs)`` creates the global variables on the ps tasks, placed
    round-robin like ``tf.train.replica_device_setter(ps_tasks)`` (worker.py:24-25).
    """

    def __init__(self, cluster, task_type="worker", task_index=0):
        self.cluster = ClusterSpec(cluster)
        self.task_type, self.task_index = task_type, int(task_index)
        self.num_ps = self.cluster.num_tasks("ps") if "ps" in self.cluster.jobs else 0
        self.num_replicas_in_sync = 1  # asynchronous: every worker applies on its own
        self.rank = self.task_index

    @classmethod
    def from_tf_config(cls, env=None):
        cluster, task_type, task_index = ClusterSpec.from_tf_config(env)
        return cls(cluster, task_type or "worker", task_index)

    @property
    def num_workers(self):
        return self.cluster.num_tasks("worker") if "worker" in self.cluster.jobs else 0

    @property
    def is_chief(self):
        return self.task_type == "worker" and self.task_index == 0

    def replica_device_setter(self):
        from .parallel.ps import replica_device_setter

        return replica_device_setter(self.num_ps, "/job:worker/task:%d" % self.task_index)

    def variable_store(self, specs, connect_timeout=120.0):
        from .parallel.ps import PSVariableStore

        return PSVariableStore(self.cluster.job_tasks("ps"), specs,
                               connect_timeout=connect_timeout,
                               setter=self.replica_device_setter())

    def run(self, fn, args=(), kwargs=None):
        return fn(*args, **(kwargs or {}))

    def reduce(self, op, value):
        return value  # no cross-worker reduction in asynchronous PS training
