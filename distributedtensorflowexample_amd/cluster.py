"""Cluster topology and per-task servers (``tf.train.ClusterSpec`` / ``Server``).

* :func:`cluster_spec` -- the reference's static localhost topology builder
  (utils.py:10-26): ps tasks on 127.0.0.1:12222.., then the workers on the
  following ports.
* :class:`ClusterSpec` -- job name -> task addresses, with TF's query API
  (``jobs``, ``num_tasks``, ``task_address``, ``job_tasks``, ``as_dict``) and
  a ``TF_CONFIG``-style environment parser.
* :class:`Server` -- ``tf.train.Server(cluster, job_name, task_index, config)``.
  A ps task hosts the native C++ parameter server (``_host.PSServer``) on its
  address (the TF gRPC server of main.py:67-68); a worker task applies its
  ``ConfigProto`` (GPU memory fraction, main.py:58-64,73) and hands out
  ``target`` -- the ps addresses a worker session connects to.
"""
from __future__ import annotations

import json
import os

from .config import ConfigProto


def cluster_spec(num_workers, num_ps, host="127.0.0.1", base_port=12222):
    """utils.py:10-26: {'ps': [host:port..], 'worker': [host:port..]}."""
    port = int(base_port)
    ps = []
    for _ in range(int(num_ps)):
        ps.append("%s:%d" % (host, port))
        port += 1
    workers = []
    for _ in range(int(num_workers)):
        workers.append("%s:%d" % (host, port))
        port += 1
    return {"ps": ps, "worker": workers}


class ClusterSpec:
    def __init__(self, cluster):
        if isinstance(cluster, ClusterSpec):
            cluster = cluster.as_dict()
        self._jobs = {}
        for job, tasks in dict(cluster).items():
            if isinstance(tasks, dict):
                self._jobs[job] = {int(k): v for k, v in tasks.items()}
            else:
                self._jobs[job] = {i: a for i, a in enumerate(tasks)}

    @property
    def jobs(self):
        return sorted(self._jobs)

    def num_tasks(self, job_name):
        return len(self._jobs[job_name])

    def task_indices(self, job_name):
        return sorted(self._jobs[job_name])

    def task_address(self, job_name, task_index):
        try:
            return self._jobs[job_name][int(task_index)]
        except KeyError:
            raise ValueError("no task %s:%s in cluster" % (job_name, task_index))

    def job_tasks(self, job_name):
        return [self._jobs[job_name][i] for i in sorted(self._jobs[job_name])]

    def as_dict(self):
        return {j: self.job_tasks(j) for j in self.jobs}

    def __eq__(self, other):
        return isinstance(other, ClusterSpec) and self.as_dict() == other.as_dict()

    def __repr__(self):
        return "ClusterSpec(%r)" % (self.as_dict(),)

    @classmethod
    def from_tf_config(cls, env=None):
        """Parse ``TF_CONFIG`` ({"cluster": {...}, "task": {"type", "index"}})."""
        cfg = json.loads((env if env is not None else os.environ.get("TF_CONFIG", "{}")) or "{}")
        task = cfg.get("task", {})
        return cls(cfg.get("cluster", {})), task.get("type"), int(task.get("index", 0))


class Server:
    """One task of the cluster.

    ps:     starts the native parameter server on its own address; ``join()``
            blocks until a client sends shutdown (the reference's
            ``while True: time.sleep(1000)``, main.py:69-70).
    worker: records the cluster and applies ``config`` (memory fraction).
    """

    def __init__(self, cluster, job_name, task_index=0, config=None, start=True):
        self.cluster = ClusterSpec(cluster)
        self.job_name = job_name
        self.task_index = int(task_index)
        self.config = config or ConfigProto()
        self.address = self.cluster.task_address(job_name, task_index)
        self._ps = None
        if start:
            self.start()

    def start(self):
        if self.job_name == "ps" and self._ps is None:
            from .ops import host

            hostname, port = self.address.rsplit(":", 1)
            self._ps = host().PSServer(hostname, int(port))
            self._ps.start()
        elif self.job_name == "worker":
            self.config.apply()

    @property
    def target(self):
        """What a worker session connects to: the ps task addresses."""
        return self.cluster.job_tasks("ps") if "ps" in self.cluster.jobs else []

    @property
    def port(self):
        return self._ps.port if self._ps is not None else int(self.address.rsplit(":", 1)[1])

    def join(self):
        if self._ps is not None:
            self._ps.join()

    def stop(self):
        if self._ps is not None:
            self._ps.stop()

    def stats(self):
        return self._ps.stats() if self._ps is not None else {}
