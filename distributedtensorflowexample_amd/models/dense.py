"""Flat-parameter dense classifiers for the async parameter-server worker.

``DenseClassifier(hidden, activation)`` is a stack of ``tf.layers.dense`` layers -- the
reference's network (worker.py:46-57) is ``DenseClassifier((100,), "sigmoid")`` -- that
*declares* its variables into a :mod:`..variables` registry (TF names ``dense/kernel``,
``dense/bias``, ``dense_1/kernel``, ... under the caller's ``variable_scope``) instead of
owning them, so the PS worker derives the ps variables, the gradient pairing, the saver's
var list and the init op from ``get_vars`` exactly as the reference does (utils.py:3-8,
worker.py:73-103).

Local replicas keep kernels in the kernels' preferred [out, in] layout (``nn.dense``: the
hand-written GEMM with fused bias + activation epilogue on the GPU); TF's [in, out] layout
exists only at the pull / push / checkpoint boundary.  The reference configuration keeps
its fused MI355X step (``ops/mlp_step.py``) -- see ``is_reference_mlp``.

``make_ps_model(name, hidden_units)``: ``mlp`` (the reference, default), ``softmax``
(softmax regression 784 -> 10: TF's MNIST-for-beginners model), or ``mlp`` with
``hidden_units`` such as ``"256,128"`` and ``activation`` relu/sigmoid.
"""
from __future__ import annotations

import torch

from .. import variables as vs
from ..ops import init as init_ops
from ..ops import nn


def _philox_kernel_init(stddev, layer):
    """N(0, stddev) kernel init drawn in the [out, in] layout with the Philox stream of
    ``models.mlp.init_params`` (offset layer << 40), returned in TF's [in, out] layout: the
    reference MLP starts from the same weights under every strategy and seed."""
    def init(shape, seed, index):
        t = torch.empty(shape[1], shape[0])
        init_ops.fill_(t, "normal", 0.0, stddev, seed=seed, offset=int(layer) << 40)
        return t.t().contiguous()
    return init


class DenseClassifier:
    def __init__(self, in_dim=784, hidden=(100,), classes=10, activation="sigmoid",
                 kernel_stddev=1.0):
        self.in_dim, self.classes = int(in_dim), int(classes)
        self.hidden = tuple(int(h) for h in hidden)
        self.activation = activation
        self.kernel_stddev = float(kernel_stddev)
        self.dims = (self.in_dim,) + self.hidden + (self.classes,)

    @property
    def is_reference_mlp(self):
        """worker.py:46-57 exactly: the fused two-launch MI355X step applies."""
        return (self.dims == (784, 100, 10) and self.activation == "sigmoid")

    @property
    def num_layers(self):
        return len(self.dims) - 1

    def build_variables(self, registry=None):
        """Declare kernel + bias of every layer in the current ``variable_scope``
        (tf.layers.dense: kernel N(0, stddev) as worker.py:51,53, bias zeros)."""
        reg = registry or vs.get_default_registry()
        out = []
        for i in range(self.num_layers):
            name = reg.unique_layer_name("dense")
            out.append(reg.get_variable(name + "/kernel", (self.dims[i], self.dims[i + 1]),
                                        initializer=_philox_kernel_init(self.kernel_stddev, i)))
            out.append(reg.get_variable(name + "/bias", (self.dims[i + 1],),
                                        initializer=vs.zeros_initializer()))
        return out

    # -- local replica (kernels [out, in]) ------------------------------------
    def new_local(self, device):
        p = []
        for i in range(self.num_layers):
            p.append(torch.zeros(self.dims[i + 1], self.dims[i], device=device))
            p.append(torch.zeros(self.dims[i + 1], device=device))
        return p

    @staticmethod
    def load_local(local, tf_values):
        """local <- TF-layout values (in trainable-variable order): the sync_op's assigns."""
        with torch.no_grad():
            for dst, src in zip(local, tf_values):
                src = torch.as_tensor(src)
                dst.copy_(src.t() if dst.dim() == 2 else src, non_blocking=True)

    def logits(self, local, x):
        h = x
        for i in range(self.num_layers):
            last = i == self.num_layers - 1
            h = nn.dense(h, local[2 * i], local[2 * i + 1], None if last else self.activation)
        return h

    def grads(self, local, x, labels):
        """Local forward/backward (worker.py:59-79): TF-layout gradients in trainable-variable
        order, mean xent loss, accuracy."""
        ps = [t.detach().requires_grad_(True) for t in local]
        loss, acc = nn.softmax_cross_entropy(self.logits(ps, x), labels)
        gs = torch.autograd.grad(loss, ps)
        out = [g.t().contiguous() if g.dim() == 2 else g.contiguous() for g in gs]
        return out, float(loss.detach()), float(acc)


def make_ps_model(name="mlp", hidden_units="", activation=None):
    name = (name or "mlp").lower()
    if name == "softmax":
        return DenseClassifier(hidden=(), activation=None)
    if name == "mlp":
        hidden = tuple(int(h) for h in str(hidden_units).split(",") if h.strip()) or (100,)
        return DenseClassifier(hidden=hidden, activation=activation or "sigmoid")
    raise ValueError("async-PS models: mlp (reference) | softmax (got %r)" % name)
