"""Asynchronous parameter-server data parallelism (between-graph replication).

The reference's only strategy: every worker keeps a local copy
of the model, pulls the global variables from the ps each step
(``sync_op``, worker.py:81-85), computes gradients locally and pushes them
to the ps, which applies them immediately with plain SGD (``train_op``,
worker.py:70-79); ``global_step`` is incremented by a separate
``AssignAdd`` (worker.py:32, 141).  Nothing synchronizes the workers, so
gradients can be stale; updates are lock-free (``use_locking=False``).

:func:`replica_device_setter` reproduces TF's placement: variables are
assigned round-robin over the ps tasks in creation order.
:class:`PSVariableStore` owns the global variables through the native C++
client (``csrc/host/ps.cpp``): create/lookup, init/assign, uninitialized
report (the Supervisor's ready_op), pull, push-and-apply, fetch-add, and the
synchronous-replicas push (:meth:`PSVariableStore.sync_push`, TF's
``SyncReplicasOptimizer``: gradients of one step are averaged over
``replicas_to_aggregate`` workers before ONE apply, stale ones dropped).
"""
from __future__ import annotations

import time

import numpy as np
import torch

from ..ops import host


def replica_device_setter(ps_tasks, worker_device=None):
    """Round-robin ps task chooser: call with the variable's creation index."""
    ps_tasks = max(1, int(ps_tasks))

    def place(index):
        return int(index) % ps_tasks

    place.ps_tasks = ps_tasks
    place.worker_device = worker_device
    return place


class PSVariableStore:
    """Global variables living on the ps job.

    ``specs``: ordered list of (name, shape, dtype) with dtype 'float32' or
    'int64'.  Float variables are exchanged through pinned host buffers.
    """

    def __init__(self, ps_addresses, specs, connect_timeout=120.0, setter=None, rpc_timeout=0.0):
        # a lost ps raises ConnectionError (host().PSConnectionLost) from any call; rpc_timeout
        # > 0 also counts a ps that stays silent that long as lost
        self.client = host().PSClient(list(ps_addresses), float(connect_timeout),
                                      float(rpc_timeout))
        self.specs = [(n, tuple(int(d) for d in s), dt) for n, s, dt in specs]
        self.setter = setter or replica_device_setter(len(ps_addresses))
        self.handles = {}
        pin = torch.cuda.is_available()
        # the float variables' pinned pull buffers are views of ONE allocation, in spec order
        # (``flat``): a worker moves a whole pull to its device with a single copy
        self._float_names = [n for n, _, dt in self.specs if dt == "float32"]
        sizes = {n: int(np.prod(s)) if s else 1 for n, s, dt in self.specs if dt == "float32"}
        self.flat = torch.empty(sum(sizes.values()), dtype=torch.float32, pin_memory=pin)
        self.bufs, off = {}, 0
        for n, s, dt in self.specs:
            if dt == "float32":
                self.bufs[n] = self.flat[off:off + sizes[n]].view(s)
                off += sizes[n]

    # -- bring-up ----------------------------------------------------------
    def create(self):
        """Chief: create every variable on its ps task (idempotent)."""
        for i, (n, s, dt) in enumerate(self.specs):
            self.handles[n] = self.client.create(n, dt, list(s), self.setter(i))
        return self

    def lookup(self, timeout=120.0, poll=0.05):
        """Non-chief: wait until the chief has created the variables."""
        t0 = time.time()
        for i, (n, s, dt) in enumerate(self.specs):
            while True:
                try:
                    self.handles[n] = self.client.lookup(n, self.setter(i))
                    break
                except RuntimeError:  # not created yet (a lost ps is a ConnectionError)
                    if time.time() - t0 > timeout:
                        raise TimeoutError("ps variable %s never created" % n)
                    time.sleep(poll)
        return self

    def uninitialized(self):
        """report_uninitialized_variables (worker.py:112-113): list of names."""
        inv = {h: n for n, h in self.handles.items()}
        return [inv[h] for h in self.client.uninitialized(list(self.handles.values()))]

    def assign(self, values):
        """Assign {name: tensor/array/int} (init or restore)."""
        for n, v in values.items():
            h = self.handles[n]
            if isinstance(v, torch.Tensor):
                v = v.detach().cpu().numpy()
            a = np.ascontiguousarray(np.asarray(v, dtype=np.float32 if n in self.bufs else np.int64))
            self.client.assign(h, a.ctypes.data, a.nbytes)

    # -- per-step traffic ---------------------------------------------------
    def pull(self, names=None):
        """Pull float variables into the pinned host buffers; returns them."""
        names = names or self._float_names
        bs = [self.bufs[n] for n in names]
        self.client.pull([self.handles[n] for n in names], [b.data_ptr() for b in bs],
                         [b.numel() * 4 for b in bs])
        return {n: b for n, b in zip(names, bs)}

    def push_apply(self, grads, lr, use_locking=False):
        """{name: contiguous f32 CPU tensor} -> var -= lr * grad on the ps."""
        names = list(grads)
        gs = [grads[n] for n in names]
        for g in gs:
            if g.dtype != torch.float32 or g.device.type != "cpu" or not g.is_contiguous():
                raise ValueError("push_apply needs contiguous f32 CPU tensors")
        self.client.push_apply([self.handles[n] for n in names], [g.data_ptr() for g in gs],
                               [g.numel() * 4 for g in gs], float(lr), bool(use_locking))

    def push_step_pull(self, grads, lr, use_locking=False, step_name="global/global_step",
                       names=None):
        """train_op + counter_op + the next step's sync_op in ONE round trip per ps task
        (pipelined requests, served in order): ``var -= lr * grad``, ``global_step += 1``,
        then the float variables pulled into the pinned buffers.  Returns (old step,
        {name: pulled tensor})."""
        gnames = list(grads)
        gs = [grads[n] for n in gnames]
        for g in gs:
            if g.dtype != torch.float32 or g.device.type != "cpu" or not g.is_contiguous():
                raise ValueError("push_step_pull needs contiguous f32 CPU tensors")
        pnames = names or self._float_names
        bs = [self.bufs[n] for n in pnames]
        old = self.client.push_step_pull(
            [self.handles[n] for n in gnames], [g.data_ptr() for g in gs],
            [g.numel() * 4 for g in gs], float(lr), bool(use_locking), self.handles[step_name],
            1, [self.handles[n] for n in pnames], [b.data_ptr() for b in bs],
            [b.numel() * 4 for b in bs])
        return int(old), {n: b for n, b in zip(pnames, bs)}

    def push_step_pull_begin(self, grads, lr, use_locking=False, step_name="global/global_step",
                             names=None):
        """Split-phase :meth:`push_step_pull`: send the push, the step increment and the pull,
        return at once (the ps works while the caller stages its next batch).  Must be
        followed by :meth:`push_step_pull_end` on the same thread (no other call on this
        store in between)."""
        gnames = list(grads)
        gs = [grads[n] for n in gnames]
        for g in gs:
            if g.dtype != torch.float32 or g.device.type != "cpu" or not g.is_contiguous():
                raise ValueError("push_step_pull needs contiguous f32 CPU tensors")
        pnames = names or self._float_names
        bs = [self.bufs[n] for n in pnames]
        self.client.push_step_pull_begin(
            [self.handles[n] for n in gnames], [g.data_ptr() for g in gs],
            [g.numel() * 4 for g in gs], float(lr), bool(use_locking), self.handles[step_name],
            1, [self.handles[n] for n in pnames], [b.data_ptr() for b in bs],
            [b.numel() * 4 for b in bs])
        self._psp_names = pnames

    def push_step_pull_end(self):
        """-> (old step, {name: pulled tensor}) of the exchange :meth:`push_step_pull_begin`
        opened."""
        old = self.client.push_step_pull_end()
        return int(old), {n: self.bufs[n] for n in self._psp_names}

    def sync_push(self, grads, lr, replicas_to_aggregate, local_step,
                  step_name="global/global_step", timeout_s=600.0):
        """Synchronous replicas (tf.train.SyncReplicasOptimizer): push this worker's
        gradients of ``local_step``; the ps accumulates them per variable and, with the
        ``replicas_to_aggregate``-th gradient of the round, applies ``var -= lr * mean`` and
        advances ``global_step``.  Blocks until the round is applied (the token queue) and
        returns ``(new_global_step, applied)``; ``applied`` is False when the gradient was
        stale (its round closed without it -- backup workers, R < num_workers) and dropped,
        as TF's ConditionalAccumulator drops it."""
        names = list(grads)
        gs = [grads[n] for n in names]
        for g in gs:
            if g.dtype != torch.float32 or g.device.type != "cpu" or not g.is_contiguous():
                raise ValueError("sync_push needs contiguous f32 CPU tensors")
        step, applied = self.client.sync_push(
            [self.handles[n] for n in names], [g.data_ptr() for g in gs],
            [g.numel() * 4 for g in gs], float(lr), int(replicas_to_aggregate), int(local_step),
            self.handles[step_name], float(timeout_s))
        return int(step), bool(applied)

    def fetch_add(self, name, delta=1):
        return int(self.client.fetch_add(self.handles[name], int(delta)))

    def read_int(self, name):
        return self.fetch_add(name, 0)

    def read_all(self):
        """{name: CPU tensor} snapshot of every variable (the chief's Saver).  Pulled into
        buffers of its own: the saver thread never writes the pull buffers the training loop
        is copying to its device."""
        names = self._float_names
        out = {n: torch.empty_like(self.bufs[n]) for n in names}
        self.client.pull([self.handles[n] for n in names], [out[n].data_ptr() for n in names],
                         [out[n].numel() * 4 for n in names])
        for n, s, dt in self.specs:
            if dt != "float32":
                out[n] = torch.tensor(self.read_int(n), dtype=torch.int32)
        return out

    def close(self):
        self.client.close()


class SyncReplicasOptimizer:
    """``tf.train.SyncReplicasOptimizer(opt, replicas_to_aggregate, total_num_replicas)`` for
    variables hosted on the ps (a :class:`PSVariableStore`).

    ``apply_gradients([(grad, name), ...])`` pushes this worker's gradients for its local
    step; the ps averages ``replicas_to_aggregate`` of them and applies ``var -= lr * mean``
    once per step (the wrapped optimizer must be a ``GradientDescentOptimizer``: the apply
    runs on the ps, like TF's ApplyGradientDescent colocated with the variables,
    worker.py:75-79).  The call blocks until the step's round is applied -- the token queue
    -- and returns the new global step, which becomes the next local step.  Gradients from a
    worker whose step was already applied (a backup replica, ``replicas_to_aggregate <
    total_num_replicas``) are dropped, as TF's accumulators drop stale gradients.
    """

    def __init__(self, opt, replicas_to_aggregate, total_num_replicas=None, store=None,
                 step_name="global/global_step", timeout_s=600.0):
        from ..optim import GradientDescentOptimizer

        if not isinstance(opt, GradientDescentOptimizer):
            raise TypeError("the ps applies plain SGD: wrap a GradientDescentOptimizer")
        if store is None:
            raise ValueError("SyncReplicasOptimizer needs the PSVariableStore of the variables")
        self.opt, self.store = opt, store
        self.replicas_to_aggregate = int(replicas_to_aggregate)
        self.total_num_replicas = int(total_num_replicas or replicas_to_aggregate)
        if self.replicas_to_aggregate < 1 or self.total_num_replicas < self.replicas_to_aggregate:
            raise ValueError("need 1 <= replicas_to_aggregate <= total_num_replicas")
        self.step_name, self.timeout_s = step_name, float(timeout_s)
        self.local_step = None
        self.dropped = 0

    def compute_gradients(self, loss, var_list):
        return self.opt.compute_gradients(loss, var_list)

    def apply_gradients(self, grads_and_vars, global_step=None):
        if self.local_step is None:
            self.local_step = self.store.read_int(self.step_name)
        grads = {name: g.detach().float().cpu().contiguous() for g, name in grads_and_vars}
        step, applied = self.store.sync_push(grads, self.opt.learning_rate,
                                             self.replicas_to_aggregate, self.local_step,
                                             self.step_name, self.timeout_s)
        self.dropped += 0 if applied else 1
        self.local_step = step
        return step
