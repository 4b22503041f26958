"""Checkpoints in TensorFlow's V2 format (``tf.train.Saver`` / ``FastSaver``).

The reference checkpoints the global variables every 30 s from the chief's
Supervisor thread with ``FastSaver`` -- a ``tf.train.Saver`` whose ``save``
forces ``write_meta_graph=False`` (utils.py:28-32, worker.py:102-103, 115):

    <logdir>/model.ckpt-<step>.index                SSTable of BundleEntryProto
    <logdir>/model.ckpt-<step>.data-00000-of-00001  raw tensor bytes
    <logdir>/checkpoint                             CheckpointState (text proto)

The bundle itself is written/read by the native C++ writer
(``csrc/host/tensor_bundle.cpp``); this module adds TF's Saver semantics:
key names (``global/dense/kernel`` ...), ``global_step`` suffixing,
``max_to_keep`` (default 5) garbage collection, the ``checkpoint`` state
file, ``latest_checkpoint`` and restore.
"""
from __future__ import annotations

import json
import os
import re
import time

import numpy as np
import torch

from ..ops import host

# TF DataType enum
_TF_DTYPE = {torch.float32: 1, torch.float64: 2, torch.int32: 3, torch.uint8: 4, torch.int16: 5,
             torch.int8: 6, torch.int64: 9, torch.bool: 10, torch.bfloat16: 14, torch.float16: 19}
_NP_OF_TF = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8,
             9: np.int64, 10: np.bool_, 19: np.float16}


def _to_cpu_tensor(v):
    if callable(v):
        v = v()
    if isinstance(v, np.ndarray):
        v = torch.from_numpy(v)
    if not isinstance(v, torch.Tensor):
        v = torch.tensor(v)
    return v.detach().to("cpu").contiguous()


def _bytes_of(t):
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().tobytes()
    return t.numpy().tobytes()


def _from_bytes(dtype, shape, raw):
    if dtype == 14:  # bfloat16
        a = np.frombuffer(raw, dtype=np.int16).copy()
        return torch.from_numpy(a).view(torch.bfloat16).reshape(shape)
    a = np.frombuffer(raw, dtype=_NP_OF_TF[dtype]).copy().reshape(shape)
    return torch.from_numpy(a)


# ---------------------------------------------------------------------------
# CheckpointState ("checkpoint" text file)
# ---------------------------------------------------------------------------
class CheckpointState:
    def __init__(self, model_checkpoint_path, all_model_checkpoint_paths):
        self.model_checkpoint_path = model_checkpoint_path
        self.all_model_checkpoint_paths = list(all_model_checkpoint_paths)


def _state_path(save_dir, latest_filename=None):
    return os.path.join(save_dir, latest_filename or "checkpoint")


def update_checkpoint_state(save_dir, model_checkpoint_path, all_model_checkpoint_paths,
                            latest_filename=None):
    def rel(p):
        return os.path.relpath(p, save_dir) if os.path.dirname(os.path.abspath(p)) == \
            os.path.abspath(save_dir) else p

    lines = ['model_checkpoint_path: "%s"' % rel(model_checkpoint_path)]
    lines += ['all_model_checkpoint_paths: "%s"' % rel(p) for p in all_model_checkpoint_paths]
    path = _state_path(save_dir, latest_filename)
    tmp = path + ".tmp%d" % os.getpid()
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, path)


def get_checkpoint_state(checkpoint_dir, latest_filename=None):
    path = _state_path(checkpoint_dir, latest_filename)
    if not os.path.exists(path):
        return None
    model, allp = None, []
    with open(path) as f:
        for line in f:
            m = re.match(r'\s*(\w+)\s*:\s*"(.*)"\s*$', line)
            if not m:
                continue
            key, val = m.group(1), m.group(2)
            if not os.path.isabs(val):
                val = os.path.join(checkpoint_dir, val)
            if key == "model_checkpoint_path":
                model = val
            elif key == "all_model_checkpoint_paths":
                allp.append(val)
    if model is None:
        return None
    return CheckpointState(model, allp or [model])


def checkpoint_exists(prefix):
    return os.path.exists(prefix + ".index")


def latest_checkpoint(checkpoint_dir, latest_filename=None):
    st = get_checkpoint_state(checkpoint_dir, latest_filename)
    if st and checkpoint_exists(st.model_checkpoint_path):
        return st.model_checkpoint_path
    return None


def load_checkpoint(prefix, verify=True):
    """{name: torch.Tensor (CPU)} of a V2 checkpoint prefix."""
    raw = host().read_bundle(prefix, verify)
    return {k: _from_bytes(dt, shape, b) for k, (dt, shape, b) in raw.items()}


def list_variables(prefix):
    raw = host().read_bundle(prefix, False)
    return sorted((k, list(shape)) for k, (dt, shape, _) in raw.items())


# ---------------------------------------------------------------------------
# Saver
# ---------------------------------------------------------------------------
class Saver:
    """Saves/restores a name -> tensor mapping in TF V2 format.

    ``var_list``: dict name -> tensor | numpy array | zero-arg callable
    returning one (callables let the saver read device-resident or
    ps-resident values at save time).  ``restore`` returns the dict of
    restored CPU tensors and, if ``assign`` was given at construction,
    calls it with that dict.
    """

    def __init__(self, var_list=None, max_to_keep=5, assign=None):
        self.var_list = dict(var_list or {})
        self.max_to_keep = max_to_keep
        self.assign = assign
        self._last = []  # [(path, time)]

    @property
    def last_checkpoints(self):
        return [p for p, _ in self._last]

    def recover_last_checkpoints(self, paths):
        self._last = [(p, time.time()) for p in paths]

    def save(self, sess=None, save_path="model.ckpt", global_step=None, latest_filename=None,
             meta_graph_suffix="meta", write_meta_graph=True, variables=None):
        values = variables if variables is not None else self.var_list
        if global_step is not None:
            if callable(global_step):
                global_step = global_step()
            if isinstance(global_step, torch.Tensor):
                global_step = int(global_step.item())
            prefix = "%s-%d" % (save_path, int(global_step))
        else:
            prefix = save_path
        save_dir = os.path.dirname(os.path.abspath(prefix))
        os.makedirs(save_dir, exist_ok=True)
        tensors = []
        for name, v in values.items():
            t = _to_cpu_tensor(v)
            if t.dtype not in _TF_DTYPE:
                raise TypeError("cannot checkpoint dtype %s (%s)" % (t.dtype, name))
            tensors.append((name, _TF_DTYPE[t.dtype], list(t.shape), _bytes_of(t)))
        host().write_bundle(prefix, tensors)
        if write_meta_graph:
            # Framework-native graph description (TF's MetaGraphDef needs TF).
            with open(prefix + "." + meta_graph_suffix + ".json", "w") as f:
                json.dump({n: list(_to_cpu_tensor(v).shape) for n, v in values.items()}, f)
        self._last = [(p, t) for p, t in self._last if p != prefix] + [(prefix, time.time())]
        self._gc(save_dir, meta_graph_suffix)
        update_checkpoint_state(save_dir, prefix, self.last_checkpoints, latest_filename)
        return prefix

    def _gc(self, save_dir, meta_suffix):
        if not self.max_to_keep:
            return
        while len(self._last) > self.max_to_keep:
            p, _ = self._last.pop(0)
            for suffix in (".index", ".data-00000-of-00001", "." + meta_suffix + ".json"):
                try:
                    os.remove(p + suffix)
                except FileNotFoundError:
                    pass

    def restore(self, sess=None, save_path=None):
        values = load_checkpoint(save_path)
        missing = [k for k in self.var_list if k not in values]
        if missing and self.var_list:
            raise KeyError("checkpoint %s lacks variables %s" % (save_path, missing))
        if self.assign is not None:
            self.assign(values)
        return values


class FastSaver(Saver):
    """utils.py:28-32 -- a Saver whose save() never writes the meta graph."""

    def save(self, sess=None, save_path="model.ckpt", global_step=None, latest_filename=None,
             meta_graph_suffix="meta", write_meta_graph=True, variables=None):
        return super().save(sess, save_path, global_step, latest_filename, meta_graph_suffix,
                            False, variables)
