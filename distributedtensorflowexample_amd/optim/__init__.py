"""TF-1.x-style optimizers (``tf.train.*Optimizer``) over the flat HIP kernels.

The reference builds ``tf.train.GradientDescentOptimizer(lr)``, calls
``compute_gradients`` and ``apply_gradients(global_step=...)`` (worker.py:71-79).
Here the same three-call API runs on torch parameters:

* ``compute_gradients(loss, var_list)`` -> ``[(grad, var), ...]`` (autograd);
* ``apply_gradients(grads_and_vars, global_step)`` -> ONE fused launch of the
  multi-tensor kernel (``csrc/kernels/optim.hip``) when the variables are
  views of one flat buffer (the framework's models and DDP allocate them that
  way), otherwise one launch per variable; ``global_step`` (an int64 tensor)
  is incremented like ``tf.train.get_or_create_global_step``;
* ``minimize(loss, ...)`` = both.

Slots (momentum / Adam moments) are allocated lazily, flat when the
variables are flat.
"""
from __future__ import annotations

import torch

from ..ops import optim as K


def _flat_base(vs):
    """If all tensors are contiguous, ordered, gap-free views of one storage, return that
    1-D span (a view) covering them; else None."""
    if not vs:
        return None
    st = vs[0].untyped_storage().data_ptr()
    if any(v.untyped_storage().data_ptr() != st or not v.is_contiguous() for v in vs):
        return None
    off = vs[0].storage_offset()
    for v in vs:
        if v.storage_offset() != off:
            return None
        off += v.numel()
    base = vs[0].untyped_storage()
    n = off - vs[0].storage_offset()
    return torch.empty(0, dtype=vs[0].dtype, device=vs[0].device).set_(
        base, vs[0].storage_offset(), (n,))


class Optimizer:
    def __init__(self, learning_rate, use_locking=False, name="Optimizer"):
        self.learning_rate = learning_rate
        self.use_locking = use_locking  # accepted for API parity; updates are stream-ordered
        self.name = name
        self._slots = {}

    # ------------------------------------------------------------------ API
    def compute_gradients(self, loss, var_list):
        grads = torch.autograd.grad(loss, var_list, allow_unused=True)
        return [(g if g is not None else torch.zeros_like(v), v) for g, v in zip(grads, var_list)]

    def apply_gradients(self, grads_and_vars, global_step=None):
        gs = [g for g, _ in grads_and_vars]
        vs = [v for _, v in grads_and_vars]
        with torch.no_grad():
            pv, pg = _flat_base(vs), _flat_base(gs)
            if pv is not None and pg is not None:
                self._apply(pv, pg, "flat")
            else:
                for i, (g, v) in enumerate(zip(gs, vs)):
                    self._apply(v.view(-1), g.contiguous().view(-1), i)
            if global_step is not None:
                global_step.add_(1)
        return global_step

    def minimize(self, loss, global_step=None, var_list=None):
        return self.apply_gradients(self.compute_gradients(loss, var_list), global_step)

    def _slot(self, key, name, like):
        k = (key, name)
        if k not in self._slots:
            self._slots[k] = torch.zeros_like(like)
        return self._slots[k]

    def _apply(self, p, g, key):  # pragma: no cover - abstract
        raise NotImplementedError


class GradientDescentOptimizer(Optimizer):
    """``var -= lr * grad`` (TF ApplyGradientDescent, worker.py:71,79)."""

    def __init__(self, learning_rate, use_locking=False, name="GradientDescent"):
        super().__init__(learning_rate, use_locking, name)

    def _apply(self, p, g, key):
        K.sgd_(p, g, self.learning_rate)


class MomentumOptimizer(Optimizer):
    def __init__(self, learning_rate, momentum, use_locking=False, name="Momentum",
                 use_nesterov=False):
        super().__init__(learning_rate, use_locking, name)
        self.momentum, self.use_nesterov = momentum, use_nesterov

    def _apply(self, p, g, key):
        # TF form: accum = momentum * accum + grad; var -= lr * accum
        K.momentum_(p, g, self._slot(key, "momentum", p), self.learning_rate, self.momentum,
                    0.0, self.use_nesterov)


class AdamOptimizer(Optimizer):
    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8,
                 use_locking=False, name="Adam", weight_decay=0.0, decoupled=True):
        super().__init__(learning_rate, use_locking, name)
        self.beta1, self.beta2, self.epsilon = beta1, beta2, epsilon
        self.weight_decay, self.decoupled = weight_decay, decoupled
        self._t = 0

    def apply_gradients(self, grads_and_vars, global_step=None):
        self._t += 1
        return super().apply_gradients(grads_and_vars, global_step)

    def _apply(self, p, g, key):
        K.adam_(p, g, self._slot(key, "m", p), self._slot(key, "v", p), self.learning_rate,
                self._t, self.beta1, self.beta2, self.epsilon, self.weight_decay, self.decoupled)


__all__ = ["Optimizer", "GradientDescentOptimizer", "MomentumOptimizer", "AdamOptimizer"]
