"""The reference's ``Worker`` (worker.py:7-159), MI355X-native.

Async parameter-server mode, with the reference's semantics step for step:

=================  =========================================  ===================
reference           here                                       native component
=================  =========================================  ===================
build_net global    ``global/dense/kernel`` ... on the ps      PSVariableStore
  (+global_step)      (round-robin over ps tasks)               (C++ PSServer)
build_net local     flat replica on the worker's GPU           fused HIP kernels
sync_op             pull -> pinned host -> H2D                 C++ PSClient
train_op            local grads (fused kernels) -> D2H ->      mlp_step kernels,
                    push + ApplyGradientDescent on the ps       C++ apply on ps
counter_op          atomic fetch_add(global_step, 1)           C++ PSServer
summary_op          loss/accuracy -> TFRecord events           C++ EventWriter
saver               FastSaver, TF V2 bundle, every 30 s        C++ bundle writer
Supervisor          chief restore-or-init, ready wait          train/supervisor.py
=================  =========================================  ===================

On a CPU-only worker (BASELINE config 1, "1 ps + 1 worker on localhost
CPU") the local forward/backward is the same math in PyTorch.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from .. import variables as vs
from ..models.dense import make_ps_model
from ..ops import mlp_step, nn
from ..parallel.ps import PSVariableStore, replica_device_setter
from ..utils.summary import FileWriter
from .saver import FastSaver
from .supervisor import Supervisor

D, H, C = mlp_step.D, mlp_step.H, mlp_step.C


def build_worker_variables(model, registry, global_scope="global", local_scope="local"):
    """worker.py:24-40: the global replica + global_step under ``global`` (on the ps), the
    local replica under ``local`` (this worker's device; never saved).  Returns the
    registry's ``get_vars('global', False)`` -- ps variables and saver var list -- and
    ``get_vars('global')`` -- the trainable ones gradients are paired with (worker.py:76-77)."""
    with registry.as_default():
        with vs.variable_scope(global_scope):
            model.build_variables()
            vs.create_global_step()
        with vs.variable_scope(local_scope):
            model.build_variables()
        return vs.get_vars(global_scope, False), vs.get_vars(global_scope)


# the reference's names (worker.py:27-31 + tf.layers.dense naming): the sync-DP checkpoints
REFERENCE_MLP_NAMES = ("global/dense/kernel", "global/dense/bias", "global/dense_1/kernel",
                       "global/dense_1/bias")
# TF-layout shapes of the fused step's flat buffer, in its order (ops/mlp_step.py)
FUSED_TF_SHAPES = ((D, H), (H,), (H, C), (C,))


def fused_tf_names(trainable):
    """Names of the fused MLP step's four TF-layout tensors, taken from the registry's
    trainable collection the way the reference pairs gradients with variables: by position
    (``zip(get_vars('global'), gvs)``, worker.py:76-77; collection order = creation order).
    Raises unless the collection is exactly the 784-100-10 kernel/bias sequence."""
    shapes = tuple(tuple(v.shape) for v in trainable)
    if shapes != FUSED_TF_SHAPES:
        raise ValueError("fused MLP layout needs trainable variables shaped %s, got %s"
                         % (FUSED_TF_SHAPES, shapes))
    return tuple(v.name for v in trainable)


def tf_vars_to_flat(v, out, names=REFERENCE_MLP_NAMES):
    """TF-layout {name: tensor} -> flat internal buffer (W stored [out, in])."""
    W1t, b1, W2t, b2 = mlp_step.unflatten(out)
    k1, c1, k2, c2 = names
    W1t.copy_(v[k1].t())
    b1.copy_(v[c1])
    W2t.copy_(v[k2].t())
    b2.copy_(v[c2])
    return out


def flat_to_tf_vars(p, names=REFERENCE_MLP_NAMES):
    W1t, b1, W2t, b2 = mlp_step.unflatten(p)
    k1, c1, k2, c2 = names
    return {k1: W1t.t(), c1: b1, k2: W2t.t(), c2: b2}


def split_tf_flat(flat, names):
    """Views of a TF-layout flat buffer (the order of ``names`` / FUSED_TF_SHAPES)."""
    out, off = {}, 0
    for k, shape in zip(names, FUSED_TF_SHAPES):
        m = 1
        for d in shape:
            m *= d
        out[k] = flat[off:off + m].view(shape)
        off += m
    return out


class Worker:
    def __init__(self, job_name, task_index, server, flags, device=None, log=print,
                 global_scope="global"):
        self.job_name = job_name
        self.task_index = int(task_index)
        self.server = server
        self.flags = flags
        self.log = log
        if device is None or device == "auto":
            device = "cuda" if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        self.is_chief = self.task_index == 0
        self.batch_size = int(flags.batch_size)
        self.lr = float(flags.learning_rate)
        # the model declares its variables; everything below is derived from the registry
        # (get_vars, utils.py:3-8) as in the reference: ps variables, gradient pairing, pull,
        # init op and the saver's var list
        self.model = make_ps_model(getattr(flags, "model", "mlp"),
                                   getattr(flags, "hidden_units", ""),
                                   getattr(flags, "activation", None))
        self.registry = vs.VariableRegistry()
        self.global_vars, self.trainable = build_worker_variables(self.model, self.registry,
                                                                  global_scope)
        self.step_name = next(v.name for v in self.global_vars if v.name.endswith("global_step"))
        self.use_fused = (self.model.is_reference_mlp and self.device.type == "cuda"
                          and 1 <= self.batch_size <= mlp_step.MAX_BATCH)
        # the fused layout's tensor names come from the registry (never literals)
        self.fused_names = (fused_tf_names(self.trainable) if self.model.is_reference_mlp
                            else None)

        # global variables on the ps (replica_device_setter(num_ps), worker.py:24-32), or with
        # --ps_device gpu in one GPU-resident store on the chief's GPU (parallel/gpu_ps.py)
        self.gpu_ps = str(getattr(flags, "ps_device", "cpu")) == "gpu"
        if self.gpu_ps:
            if not self.use_fused:
                raise ValueError("--ps_device gpu needs the reference MLP on a GPU worker and "
                                 "1 <= batch_size <= %d" % mlp_step.MAX_BATCH)
            if bool(getattr(flags, "sync_replicas", False)):
                raise ValueError("--sync_replicas runs on the TCP parameter server "
                                 "(--ps_device cpu)")
            from ..parallel.gpu_ps import GpuPSStore

            self.store = GpuPSStore(server.target, self.device, int(flags.num_workers),
                                    setter=replica_device_setter(len(server.target)))
        else:
            self.store = PSVariableStore(server.target, [v.spec for v in self.global_vars],
                                         setter=replica_device_setter(len(server.target)),
                                         rpc_timeout=float(getattr(flags, "ps_timeout_secs", 0)
                                                           or 0))
        # local replica (worker.py:34-40): the fused MLP keeps one flat buffer on this
        # worker's device; other models a list of [out, in] kernels / biases
        if self.use_fused:
            self.params = torch.zeros(mlp_step.NPARAM, device=self.device)
            self.grad = torch.zeros_like(self.params)
            self.ws = mlp_step.StepWorkspace(self.batch_size, self.device)
            self.xb = torch.empty(self.batch_size, D, device=self.device)
            self.yb = torch.empty(self.batch_size, dtype=torch.int32, device=self.device)
            # the gradient leaves the GPU already in TF layout (transposed on the device) plus
            # the step's loss / accuracy record: ONE D2H copy per step into pinned memory
            n = mlp_step.NPARAM
            self._gtf_dev = torch.empty(n + 2, device=self.device)
            self.grad_host = torch.empty(n + 2, pin_memory=True)
            self._xs = torch.empty(self.batch_size, D, pin_memory=True)
            self._ys = torch.empty(self.batch_size, dtype=torch.int32, pin_memory=True)
            self._rec = None  # host mirror of the kernels' step counter (stats ring slot)
            self._staged = False  # a batch staged by stage() and not consumed yet
            # parameters of the last exchange waiting in the store's pinned pull buffer: the
            # next compute() lands them (H2D + layout) in the same native call as its step
            self._pull_pending = False
            self._pull_dev = torch.empty(mlp_step.NPARAM, device=self.device)
        else:
            self.local = self.model.new_local(self.device)
        self._test = None  # device-resident test set of the eval op (uploaded once)
        self.summary_writer = FileWriter(flags.logdir + "_%d" % self.task_index)
        # FastSaver over get_vars('global', False) (worker.py:102-103)
        self.saver = FastSaver({v.name: None for v in self.global_vars}, assign=self.store.assign)

    # -- graph pieces (as ops) ---------------------------------------------
    def init_op(self):
        """global_init_op over get_vars('global', False) (worker.py:98-99): kernels
        N(0, 1), biases 0, global_step 0 -- each variable's declared initializer."""
        seed = int(getattr(self.flags, "seed", 0))
        self.store.assign({v.name: (0 if v.dtype != "float32" else v.initial_value(seed, i))
                           for i, v in enumerate(self.global_vars)})

    def sync_op(self):
        """worker.py:81-85: local <- global for every trainable variable."""
        self._assign_local(self.store.pull())
        self._land_pull()  # the explicit sync op lands at once (the fused RPC path defers)

    def _assign_local(self, vals):
        with torch.no_grad():
            flat = getattr(self.store, "flat", None)
            if (self.use_fused and flat is not None and flat.numel() == mlp_step.NPARAM
                    and flat.is_pinned()
                    and all(vals[k].data_ptr() == self.store.bufs[k].data_ptr() for k in vals)):
                # the pull landed in the store's one pinned buffer (TF layout, spec order): the
                # next compute() copies + converts it in its native call (_land_pull otherwise)
                self._pull_pending = True
            elif self.use_fused:
                dev = {k: t.to(self.device, non_blocking=True) for k, t in vals.items()}
                tf_vars_to_flat(dev, self.params, self.fused_names)
            else:
                self.model.load_local(self.local, [vals[v.name] for v in self.trainable])

    def _land_pull(self):
        """Apply a pending pull to the device parameters now (one H2D + one layout kernel):
        before anything but compute() reads ``self.params``."""
        if self.use_fused and self._pull_pending:
            self._pull_dev.copy_(self.store.flat, non_blocking=True)
            mlp_step.from_tf_layout(self._pull_dev, self.params)
            self._pull_pending = False

    def stage(self, batch_x, batch_y):
        """Fused GPU worker: the batch -> pinned staging buffers -> asynchronous H2D into the
        device batch (one native call).  Called while the previous step's push/pull is in
        flight on the ps (``push_step_pull_begin``), so the host copy and the transfer leave the
        critical path.  The staging buffers are free: every compute ends with a stream wait
        that covers their last H2D."""
        if not (self.use_fused and batch_x.shape[0] == self.batch_size):
            return False
        from ..ops._ext import hip, ptr, stream_handle

        y = np.asarray(batch_y)
        self._xs.numpy()[...] = batch_x
        self._ys.numpy()[...] = y.argmax(1) if y.ndim == 2 else y
        hip().mlp_ps_stage(ptr(self._xs), ptr(self._ys), ptr(self.xb), ptr(self.yb),
                           self.batch_size, stream_handle(self.device))
        self._staged = True
        return True

    def compute(self, batch_x, batch_y, staged=False):
        """Local forward/backward -> (grads {global name: TF-layout CPU tensor}, loss,
        accuracy): the reference's zip(get_vars('global'), local gradients) pairing.
        ``staged``: the batch is already on its way to the device (:meth:`stage`)."""
        y = np.asarray(batch_y)
        labels = y.argmax(1) if y.ndim == 2 else y
        if self.use_fused and batch_x.shape[0] == self.batch_size:
            from ..ops._ext import hip, ptr, stream_handle

            if not (staged and self._staged):
                self.stage(batch_x, batch_y)
            self._staged = False
            rec = self.ws.global_step() if self._rec is None else self._rec
            self._rec = rec + 1
            n = mlp_step.NPARAM
            ws = self.ws
            # ONE native call: batch + pulled parameters in, forward/backward, the TF-layout
            # gradient + this step's loss / accuracy record out, stream wait (GIL released)
            hip().mlp_ps_worker_step(
                ptr(self.params), ptr(self.store.flat) if self._pull_pending else 0,
                ptr(self._pull_dev), 0, 0, ptr(self.xb), ptr(self.yb),  # batch: staged
                ptr(self.grad), ptr(ws.buf), ptr(ws.ctr), ptr(ws.stats), ws.stats_ring,
                ptr(ws.stats) + 8 * (rec % ws.stats_ring), self.batch_size, ptr(self._gtf_dev),
                ptr(self.grad_host), stream_handle(self.device))
            self._pull_pending = False
            loss, acc = self.grad_host[n:n + 2].tolist()
            return split_tf_flat(self.grad_host, self.fused_names), float(loss), float(acc)
        elif self.use_fused or self.model.is_reference_mlp:
            x = torch.from_numpy(np.ascontiguousarray(batch_x, np.float32))
            self._land_pull()
            p = self.params.cpu() if hasattr(self, "params") else self._flat_local()
            g, loss_t, acc_t = mlp_step.reference_step(p, x, torch.from_numpy(labels))
            loss, acc = float(loss_t), float(acc_t)
        else:
            x = torch.from_numpy(np.ascontiguousarray(batch_x, np.float32)).to(self.device)
            lab = torch.from_numpy(labels.astype(np.int64)).to(self.device)
            gs, loss, acc = self.model.grads(self.local, x, lab)
            return ({v.name: t.cpu().contiguous() for v, t in zip(self.trainable, gs)},
                    float(loss), float(acc))
        tfg = {k: t.contiguous() for k, t in flat_to_tf_vars(g.cpu(), self.fused_names).items()}
        return tfg, float(loss), float(acc)

    def _flat_local(self):
        """Reference MLP on a non-fused device: the local replica as the flat layout."""
        p = torch.empty(mlp_step.NPARAM)
        W1t, b1, W2t, b2 = mlp_step.unflatten(p)
        for dst, src in zip((W1t, b1, W2t, b2), self.local):
            dst.copy_(src)
        return p

    def compute_device(self, batch_x, batch_y):
        """Local forward/backward with the gradient left in ``self.grad`` on the device (GPU
        parameter store: nothing crosses to the host but the loss / accuracy record).  The
        batch goes through pinned staging buffers (asynchronous H2D), and the record's ring
        slot comes from a host mirror of the kernel's step counter (no read-back)."""
        if self._rec is None:
            self._rec = self.ws.global_step()
        y = np.asarray(batch_y)
        labels = y.argmax(1) if y.ndim == 2 else y
        torch.cuda.current_stream(self.device).synchronize()  # staging free (previous copy)
        self._xs.numpy()[...] = batch_x
        self._ys.numpy()[...] = labels
        self.xb.copy_(self._xs, non_blocking=True)
        self.yb.copy_(self._ys, non_blocking=True)
        mlp_step.step_grad(self.params, self.xb, self.yb, self.ws, self.grad)
        self._rec_slot = self._rec % self.ws.stats_ring
        self._rec += 1

    def step_record(self):
        """(loss, accuracy) the last compute_device step recorded on the device."""
        loss, acc = self.ws.stats[self._rec_slot].tolist()
        return float(loss), float(acc)

    def accuracy(self, images, labels):
        """worker.py:87-90,150-154 on the local replica: the 10k-image test accuracy.  The
        test set is uploaded once and stays resident; on the GPU the forward is the
        hand-written GEMM with the bias + sigmoid epilogue fused (nn.gemm / nn.dense)."""
        if self._test is None or self._test[0] is not images:
            x = torch.from_numpy(np.ascontiguousarray(images, np.float32)).to(self.device)
            y = np.asarray(labels)
            y = torch.from_numpy(y.argmax(1) if y.ndim == 2 else y).to(self.device)
            self._test = (images, x, y)
        _, x, y = self._test
        self._land_pull()
        with torch.no_grad():
            if self.use_fused:
                W1t, b1, W2t, b2 = mlp_step.unflatten(self.params)
                h = nn.gemm(x, W1t, trans_b=True, bias=b1, act="sigmoid")
                logits = nn.gemm(h, W2t, trans_b=True, bias=b2)
            else:
                logits = self.model.logits(self.local, x)
            return float((logits.argmax(1) == y).float().mean())

    def graph_def(self):
        """The reference graph over this worker's registry variables (utils/graph.py), or None
        for models without the reference MLP's layer structure."""
        if len(self.trainable) % 2:
            return None
        from ..utils.graph import reference_mlp_graph

        return reference_mlp_graph(self.global_vars, self.trainable, self.task_index,
                                   learning_rate=self.lr)

    # -- training loop (worker.py:105-159) ------------------------------------
    def learn(self, dataset, max_steps=None, stop_after_secs=None):
        try:
            return self._learn(dataset, max_steps, stop_after_secs)
        finally:
            if self.gpu_ps:  # also on an exception: peers must not outlive the owner's store
                self.store.close()  # the chief frees it once every other worker detached

    def _learn(self, dataset, max_steps=None, stop_after_secs=None):
        fl = self.flags
        sv = Supervisor(is_chief=self.is_chief, logdir=fl.logdir, saver=self.saver,
                        summary_writer=self.summary_writer, ready_op=self.store.uninitialized,
                        global_step=lambda: self.store.read_int(self.step_name),
                        save_model_secs=getattr(fl, "save_model_secs", 30),
                        save_summaries_secs=getattr(fl, "save_summaries_secs", 30),
                        init_op=self.init_op, local_init_op=None,
                        recovery_wait_secs=1.0, save_variables=self.store.read_all,
                        graph=self.graph_def())
        if self.is_chief:
            self.store.create()
        else:
            self.store.lookup()
        sync = bool(getattr(fl, "sync_replicas", False))
        replicas = 0
        if sync:  # default: one gradient from every worker per round
            replicas = (int(getattr(fl, "replicas_to_aggregate", 0) or 0)
                        or int(getattr(fl, "num_workers", 1)))
        log_every = int(getattr(fl, "log_every", 100))
        eval_every = int(getattr(fl, "eval_every", 10000))
        local_steps = 0
        history = []
        t_begin = time.time()
        with sv.managed_session(self.server.target):
            start_time = time.time()
            start_step = 0
            # --sync_replicas (TF's SyncReplicasOptimizer): this worker's local step is the
            # global step it read; each push joins that step's round on the ps, which applies
            # the mean of replicas_to_aggregate gradients and advances global_step
            local_step = self.store.read_int(self.step_name) if sync else 0
            fused_rpc = bool(getattr(fl, "ps_fused_rpc", True)) and not self.gpu_ps
            pulled = False  # the parameters for the next step already came with the last push
            next_gen_check = time.time() + 0.5
            nxt = None  # the next batch, drawn (and staged) during the last exchange
            split_rpc = hasattr(self.store, "push_step_pull_begin")
            while not sv.should_stop():
                if self.gpu_ps:
                    # the same four ops on the device, stream-ordered: pull (peer read), local
                    # forward/backward, remote ApplyGradientDescent (peer read-modify-write),
                    # AssignAdd on global_step (system-scope atomic; returns the old value)
                    self.store.pull_into(self.params)
                    batch_x, batch_y = dataset.train.next_batch(self.batch_size)
                    self.compute_device(batch_x, batch_y)
                    self.store.push_apply_flat(self.grad, self.lr,
                                               bool(getattr(fl, "use_locking", False)))
                    # counter_op + the step's loss / accuracy record: one read-back
                    step, (cost, acc) = self.store.fetch_add_record(
                        self.ws.stats[self._rec_slot])
                    self.summary_writer.add_scalars({"loss": cost, "accuracy": acc}, step)
                    history.append((step, cost, acc))
                    local_steps += 1
                    now = time.time()
                    if now >= next_gen_check:  # the chief's store was not replaced: checked on
                        next_gen_check = now + 0.5  # a time interval (one ps RPC), not a step count
                        self.store.check_generation()
                    if step % log_every == 0 and step != 0:
                        elapsed = time.time() - start_time
                        self.log("step: {}\t| cost: {}\t| speed: {}step/sec".format(
                            step, cost, float((step - start_step) / max(elapsed, 1e-9))))
                        start_time = time.time()
                        start_step = step
                    if step % eval_every == 0:
                        self.log("test accuracy: {}".format(
                            self.accuracy(dataset.test.images, dataset.test.labels)))
                    if step >= fl.training_steps:
                        break
                    if max_steps is not None and local_steps >= max_steps:
                        break
                    if stop_after_secs is not None and time.time() - t_begin > stop_after_secs:
                        break
                    continue
                if not pulled:
                    self.sync_op()
                if nxt is None:
                    batch_x, batch_y = dataset.train.next_batch(self.batch_size)
                    staged = False
                else:
                    (batch_x, batch_y), staged, nxt = nxt, True, None
                grads, cost, acc = self.compute(batch_x, batch_y, staged=staged)
                if sync:
                    step = local_step
                    local_step, _ = self.store.sync_push(grads, self.lr, replicas, local_step)
                elif fused_rpc and split_rpc:
                    # train_op, counter_op and the NEXT step's sync_op in one round trip
                    # (pipelined on the ps connection, served in the reference's order),
                    # split in two: the next batch is drawn and staged to the device while
                    # the ps applies / counts / reads.  Per-worker order stays pull ->
                    # compute -> push -> step (worker.py:129-141)
                    self.store.push_step_pull_begin(
                        grads, self.lr, bool(getattr(fl, "use_locking", False)), self.step_name)
                    try:
                        nxt = dataset.train.next_batch(self.batch_size)
                        self.stage(*nxt)
                    finally:
                        step, vals = self.store.push_step_pull_end()
                    self._assign_local(vals)
                    pulled = True
                elif fused_rpc:
                    step, vals = self.store.push_step_pull(
                        grads, self.lr, bool(getattr(fl, "use_locking", False)), self.step_name)
                    self._assign_local(vals)
                    pulled = True
                else:
                    self.store.push_apply(grads, self.lr, bool(getattr(fl, "use_locking", False)))
                    step = self.store.fetch_add(self.step_name, 1)  # counter_op; old value
                self.summary_writer.add_scalars({"loss": cost, "accuracy": acc}, step)
                history.append((step, cost, acc))
                local_steps += 1
                if step % log_every == 0 and step != 0:
                    elapsed = time.time() - start_time
                    self.log("step: {}\t| cost: {}\t| speed: {}step/sec".format(
                        step, cost, float((step - start_step) / max(elapsed, 1e-9))))
                    start_time = time.time()
                    start_step = step
                if step % eval_every == 0:
                    self.log("test accuracy: {}".format(
                        self.accuracy(dataset.test.images, dataset.test.labels)))
                if step >= fl.training_steps:
                    break
                if max_steps is not None and local_steps >= max_steps:
                    break
                if stop_after_secs is not None and time.time() - t_begin > stop_after_secs:
                    break
        return history
