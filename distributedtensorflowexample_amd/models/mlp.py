"""The reference model: 784 -> dense(100, sigmoid) -> dense(10) -> softmax.

worker.py:46-57 (``build_net``) with ``tf.random_normal_initializer()``
kernels (mean 0, stddev 1) and ``tf.layers.dense``'s zero bias init, and the
loss of worker.py:59-68.

All four parameters are views into ONE flat f32 buffer laid out as the fused
step kernels expect (``ops/mlp_step.py``)::

    W1t [100][784] | b1 [100] | W2t [10][100] | b2 [10]

W1t/W2t are stored [out, in]; checkpoints expose TF's [in, out] kernels
under TF's variable names (``VARIABLE_NAMES``), so a saved model has the keys
of worker.py:27-31 (``global/dense/kernel`` ...).
"""
from __future__ import annotations

import torch

from ..ops import init as init_ops
from ..ops import mlp_step, nn

D, H, C = mlp_step.D, mlp_step.H, mlp_step.C

# TF names of the global-scope variables of worker.py:27-31 (tf.layers.dense
# default naming), with their TF shapes.  ``global_step`` is int32 [].
VARIABLE_NAMES = (
    ("dense/kernel", (D, H)),
    ("dense/bias", (H,)),
    ("dense_1/kernel", (H, C)),
    ("dense_1/bias", (C,)),
)


def init_params(device="cpu", seed=0, stddev=1.0):
    """Flat parameter buffer initialised like the reference (W ~ N(0, 1), b = 0)."""
    p = torch.zeros(mlp_step.NPARAM, device=device, dtype=torch.float32)
    W1t, b1, W2t, b2 = mlp_step.unflatten(p)
    init_ops.fill_(W1t, "normal", 0.0, stddev, seed=seed, offset=0)
    init_ops.fill_(W2t, "normal", 0.0, stddev, seed=seed, offset=1 << 40)
    return p


def to_tf_variables(p):
    """{tf_name: tensor in TF layout} for checkpoints/summaries (copies to CPU)."""
    W1t, b1, W2t, b2 = (t.detach().cpu() for t in mlp_step.unflatten(p))
    return {
        "dense/kernel": W1t.t().contiguous(),
        "dense/bias": b1.clone(),
        "dense_1/kernel": W2t.t().contiguous(),
        "dense_1/bias": b2.clone(),
    }


def from_tf_variables(p, variables):
    """Load TF-layout tensors into the flat buffer (inverse of ``to_tf_variables``)."""
    W1t, b1, W2t, b2 = mlp_step.unflatten(p)
    with torch.no_grad():
        W1t.copy_(torch.as_tensor(variables["dense/kernel"]).t())
        b1.copy_(torch.as_tensor(variables["dense/bias"]))
        W2t.copy_(torch.as_tensor(variables["dense_1/kernel"]).t())
        b2.copy_(torch.as_tensor(variables["dense_1/bias"]))
    return p


class MnistMLP(torch.nn.Module):
    """Autograd module over the flat buffer (generic, eager path).

    Uses the fused-epilogue dense kernel and the fused softmax-xent kernel on
    the GPU; the same math in PyTorch on the CPU.  The flat buffer is shared
    with ``FusedMLPTrainer`` so both paths see the same parameters.
    """

    def __init__(self, device="cpu", seed=0, flat=None):
        super().__init__()
        flat = init_params(device, seed) if flat is None else flat
        self.flat = torch.nn.Parameter(flat)

    def parameters_tf(self):
        return to_tf_variables(self.flat.data)

    def views(self):
        return mlp_step.unflatten(self.flat)

    def forward(self, x):
        """Returns (softmax probabilities, logits) like build_net (worker.py:46-57)."""
        W1t, b1, W2t, b2 = self.views()
        h = nn.dense(x, W1t, b1, "sigmoid")
        logits = nn.dense(h, W2t, b2, None)
        return torch.softmax(logits, dim=-1), logits

    def loss(self, x, labels):
        """(mean xent, accuracy) of worker.py:59-68 / 87-90."""
        _, logits = self.forward(x)
        return nn.softmax_cross_entropy(logits, labels)
