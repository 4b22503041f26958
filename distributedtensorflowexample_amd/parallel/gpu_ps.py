"""GPU-resident parameter store for the async-PS mode (``--ps_device gpu``).

The reference keeps its global variables on the ps task (``replica_device_setter``,
worker.py:24-32) and moves them over gRPC every step: a pull of 318 KB (worker.py:131), a
push + remote ``ApplyGradientDescent`` (worker.py:79,135-137) and an ``AssignAdd`` on
``global_step`` (worker.py:32,141).  This store keeps the same variables -- same TF names,
same semantics (lock-free apply unless ``use_locking``, ``fetch_add`` returning the old step)
-- in ONE uncached allocation on the chief worker's GPU (``csrc/kernels/gpu_ps.cpp``); every
other worker maps it over IPC, so a pull is a peer read and an apply a peer read-modify-write
over xGMI, issued from the worker's own stream with no host copy of parameters or gradients.

The TCP parameter server stays the control plane only: it carries the allocation's IPC handle,
a detach counter (the owner frees the memory only after every other worker detached, so
no peer is ever left with a dangling mapping; a peer that never detaches within the close
timeout leaves the allocation alive until the owner's process exits) and a store generation.

Failure semantics differ from the reference's in one respect: the variables live in the
CHIEF's process, not on the ps task, so a chief failure loses them (a restarted chief
restores the last checkpoint into a NEW store).  The chief bumps the generation at every
``create()``; the other workers compare it periodically (``check_generation``) and exit
non-zero instead of training on a stale mapping.  Checkpoint / restore / readiness read and
write the GPU store (``read_all`` / ``assign`` / ``uninitialized``), so the Supervisor and
Saver work unchanged.

Internal layout: the flat MLP buffer of ``ops/mlp_step.py`` (W1 stored [out, in]); TF layouts
are converted at the ``assign`` / ``pull`` / ``read_all`` boundary.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from ..ops import mlp_step
from ..ops._ext import hip, stream_handle
from .ps import PSVariableStore

HANDLE = "gpu_ps/ipc_handle"
DETACHED = "gpu_ps/detached"
GENERATION = "gpu_ps/generation"
STEP_SLOT, INIT_SLOT = 0, 1


def _flat_from_tf(values, out):
    W1t, b1, W2t, b2 = mlp_step.unflatten(out)
    W1t.copy_(torch.as_tensor(values["global/dense/kernel"]).t())
    b1.copy_(torch.as_tensor(values["global/dense/bias"]))
    W2t.copy_(torch.as_tensor(values["global/dense_1/kernel"]).t())
    b2.copy_(torch.as_tensor(values["global/dense_1/bias"]))
    return out


def _tf_from_flat(p):
    W1t, b1, W2t, b2 = mlp_step.unflatten(p)
    return {"global/dense/kernel": W1t.t().contiguous(), "global/dense/bias": b1.clone(),
            "global/dense_1/kernel": W2t.t().contiguous(), "global/dense_1/bias": b2.clone()}


class GpuPSStore:
    """Drop-in for ``PSVariableStore`` (the MLP's GLOBAL_SPECS) with the variables in GPU
    memory.  ``create()`` (chief) allocates on ``device``; ``lookup()`` (other workers) opens
    the chief's allocation.  Fast path: ``pull_into`` / ``push_apply_flat`` on device
    buffers."""

    STEP = "global/global_step"

    def __init__(self, ps_addresses, device, num_workers, setter=None, connect_timeout=120.0):
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("GpuPSStore needs a GPU device")
        self.num_workers = int(num_workers)
        nbytes = hip().GpuParamStore.handle_size()
        self._hwords = nbytes // 4
        self.ctl = PSVariableStore(ps_addresses, [(HANDLE, (self._hwords,), "float32"),
                                                  (DETACHED, (), "int64"),
                                                  (GENERATION, (), "int64")],
                                   connect_timeout=connect_timeout, setter=setter)
        self.generation = None
        self._kept_alive = None  # an allocation a peer never detached from (owner)
        self.n = mlp_step.NPARAM
        self._st = None
        self._owner = False
        self._host = torch.empty(self.n, dtype=torch.float32, pin_memory=True)

    # -- bring-up -----------------------------------------------------------
    def create(self):
        """Chief: allocate the store on this GPU and publish its IPC handle."""
        self.ctl.create()
        self._st = hip().GpuParamStore(self.device.index or 0, self.n, True)
        self._owner = True
        h = np.frombuffer(self._st.handle(), dtype=np.float32).copy()
        self.ctl.assign({DETACHED: 0})
        if GENERATION in self.ctl.uninitialized():  # first store of this ps
            self.ctl.assign({GENERATION: 1})
            self.generation = 1
        else:  # a restarted chief: a new store generation
            self.generation = self.ctl.fetch_add(GENERATION, 1) + 1
        self.ctl.assign({HANDLE: torch.from_numpy(h)})
        return self

    def lookup(self, timeout=120.0, poll=0.05):
        """Non-chief: wait for the chief's handle, then map the store."""
        self.ctl.lookup(timeout=timeout, poll=poll)
        t0 = time.time()
        while True:
            if not self.ctl.uninitialized():
                h = self.ctl.pull([HANDLE])[HANDLE].numpy().tobytes()
                if any(h):
                    break
            if time.time() - t0 > timeout:
                raise TimeoutError("gpu_ps: the chief never published the store")
            time.sleep(poll)
        self.generation = self.ctl.read_int(GENERATION)
        self._st = hip().GpuParamStore(self.device.index or 0, self.n, False)
        self._st.open(h)
        return self

    def check_generation(self):
        """Non-chief: raise if the chief re-created the store since ``lookup`` (its process
        restarted: this worker's mapping no longer holds the global variables)."""
        if self._owner or self.generation is None:
            return
        g = self.ctl.read_int(GENERATION)
        if g != self.generation:
            raise RuntimeError("gpu_ps: the chief re-created the parameter store (generation "
                               "%d -> %d); this worker's mapping is stale" % (self.generation, g))

    def _ctrl(self, slot, delta):
        return int(self._st.fetch_add(slot, int(delta), stream_handle(self.device)))

    def uninitialized(self):
        """report_uninitialized_variables: every variable until the first assign."""
        if self._st is None or self._ctrl(INIT_SLOT, 0) == 0:
            return ["global/dense/kernel", "global/dense/bias", "global/dense_1/kernel",
                    "global/dense_1/bias", self.STEP]
        return []

    def assign(self, values):
        """Init / restore: {TF name: tensor/array/int}; the float variables are assigned
        together (all four are required), global_step alone is allowed."""
        floats = [k for k in values if k != self.STEP]
        if floats:
            if len(floats) != 4:
                raise ValueError("gpu_ps: assign all four float variables together")
            _flat_from_tf(values, self._host)
            self._st.write(self._host.data_ptr(), 0, self.n * 4)
        if self.STEP in values:
            s = int(torch.as_tensor(values[self.STEP]).item())
            cur = self._ctrl(STEP_SLOT, 0)
            self._ctrl(STEP_SLOT, s - cur)
        if self._ctrl(INIT_SLOT, 0) == 0:
            self._ctrl(INIT_SLOT, 1)

    # -- per-step traffic -----------------------------------------------------
    def pull_into(self, dst):
        """sync_op on the device: dst (flat f32 [NPARAM] on this GPU) <- store."""
        self._st.pull(dst.data_ptr(), stream_handle(self.device))

    def push_apply_flat(self, grad, lr, use_locking=False):
        """ApplyGradientDescent on the store from a flat device gradient (stream-ordered)."""
        self._st.push_apply(grad.data_ptr(), float(lr), bool(use_locking),
                            stream_handle(self.device))

    def pull(self, names=None):
        host = torch.empty(self.n, dtype=torch.float32, pin_memory=True)  # saver thread too
        self._st.read(host.data_ptr(), 0, self.n * 4)
        v = _tf_from_flat(host)
        return {k: v[k] for k in (names or v)}

    def push_apply(self, grads, lr, use_locking=False):
        g = _flat_from_tf(grads, torch.zeros(self.n, dtype=torch.float32)).to(self.device)
        self.push_apply_flat(g, lr, use_locking)
        torch.cuda.synchronize(self.device)

    def sync_push(self, *a, **k):
        raise NotImplementedError("--sync_replicas runs on the TCP parameter server "
                                  "(--ps_device cpu)")

    def fetch_add(self, name, delta=1):
        if name != self.STEP:
            raise KeyError(name)
        return self._ctrl(STEP_SLOT, delta)

    def fetch_add_record(self, record, delta=1):
        """global_step fetch-add that also reads back ``record`` (a small f32 device tensor:
        the step's loss / accuracy) in the same copy -- one host round trip per step."""
        old, vals = self._st.fetch_add_read(STEP_SLOT, int(delta), stream_handle(self.device),
                                            record.data_ptr(), record.numel())
        return int(old), vals

    def read_int(self, name):
        return self.fetch_add(name, 0)

    def read_all(self):
        out = self.pull()
        out[self.STEP] = torch.tensor(self.read_int(self.STEP), dtype=torch.int32)
        return out

    def close(self, timeout=60.0, poll=0.05):
        """Detach (non-owner) or wait for every other worker to detach, then free (owner).

        Owner: once the wait ends the published handle is cleared BEFORE anything is freed,
        so a worker that looks the store up later fails cleanly instead of mapping memory
        about to be freed (one that joins during the wait trains and detaches).  If some peer has not
        detached within ``timeout`` seconds the allocation is NOT freed (a peer may still be
        pulling or applying through its mapping): it stays alive until this process exits,
        with a warning."""
        if self._st is None:
            return
        torch.cuda.synchronize(self.device)
        if self._owner:
            t0 = time.time()
            while (self.ctl.read_int(DETACHED) < self.num_workers - 1
                   and time.time() - t0 < timeout):
                time.sleep(poll)
            # late lookups from here on find no handle and fail cleanly
            self.ctl.assign({HANDLE: torch.zeros(self._hwords)})
            missing = self.num_workers - 1 - self.ctl.read_int(DETACHED)
            if missing > 0:
                import warnings

                warnings.warn("gpu_ps: %d worker(s) never detached within %.0f s; the store "
                              "stays allocated until this process exits" % (missing, timeout))
                self._kept_alive = self._st
            else:
                self._st.close()
        else:
            self._st.close()
            self.ctl.fetch_add(DETACHED, 1)
        self._st = None
