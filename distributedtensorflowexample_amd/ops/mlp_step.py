"""Fused three-launch training step of the reference MNIST MLP.

Python side of ``csrc/kernels/mlp_step.hip``; see that file for the kernel
design.  The step the reference runs per worker (worker.py:131-141: pull,
forward, loss, backward, ApplyGradientDescent, global_step += 1) becomes::

    mlp_fwd   : partial z1 = x . W1 over 7 K slices (343 single-wave blocks)
    mlp_head  : per-row sigmoid, logits, softmax-xent, accuracy, dlogits, dz1
    mlp_wgrad : dW1, dW2, db1, db2 (+ the SGD apply fused in, single GPU)

Sync data-parallel mode instead writes the flat gradient, all-reduces it and
applies it at the start of the next step (``mlp_fwd``/``mlp_head`` with
``grad``/``p_new``: deferred apply into a ping-pong parameter buffer).

Flat parameter layout (shared with gradients and all-reduce buckets)::

    W1t [100][784] | b1 [100] | W2t [10][100] | b2 [10]      (79,510 f32)

``reference_step`` is the same math in plain PyTorch (float64-capable), the
numerics oracle of the kernel tests and the CPU path of the PS worker.
"""
from __future__ import annotations

import os

import torch

from ._ext import hip, ptr, stream_handle

D, H, C = 784, 100, 10
HT, HP = 7, 112
OFF_W1 = 0
OFF_B1 = OFF_W1 + H * D
OFF_W2 = OFF_B1 + H
OFF_B2 = OFF_W2 + C * H
NPARAM = OFF_B2 + C
MAX_BATCH = 256


# partial z1 slabs the data-parallel engines' first launch writes (their K slicing)
XG_SLABS = 28
# 16-byte LL layout of the fused engines' one-shot split exchange (csrc/kernels/mlp_step.hip,
# xg_exchange16): a communicator for fused2 needs slots of XG_SLOT_WORDS words
XG_W1_BASE = 79616
XG_SLOT_WORDS = XG_W1_BASE + 7 * 28 * 2 * 2 * 64 * 2
# z1 slabs of the factor engines' first launch (mlp_fwdapply_factor_kernel's K slicing)
FACTOR_SLABS = 28


def engine_slot_words(kind):
    """Words per slot of a data-parallel engine's communicator: the pipelined fused engines'
    W1 exchange (one-shot fused2, two-shot fused2x) moves 16-byte word pairs in a layout past
    the parameter-offset region (XG_SLOT_WORDS); the others exchange at parameter offsets."""
    return XG_SLOT_WORDS if kind in ("fused2", "fused2x") else NPARAM


def xg_w1_pair_offsets():
    """Slot word offset of every W1 element (flat [100][784] order) in the 16-byte layout:
    element (hidden j, feature f) is lane (4 q + ..) r of K-split wave sp = i // 2 of column
    group cgp of block (jt, ks), word e = i % 2 of its pair (j = 16 jt + 4 q + i, f = 28 ks +
    16 cgp + r)."""
    j = torch.arange(H).view(H, 1).expand(H, D)
    f = torch.arange(D).view(1, D).expand(H, D)
    jt, hl = j // 16, j % 16
    q, i = hl // 4, hl % 4
    ks, fl = f // 28, f % 28
    cgp, r = fl // 16, fl % 16
    eslot = (jt * 28 + ks) * 2 + cgp
    sp, e = i // 2, i % 2
    lane = q * 16 + r
    return (XG_W1_BASE + ((eslot * 2 + sp) * 64 + lane) * 2 + e).reshape(-1)

def unflatten(p):
    """Views (W1t [H,D], b1 [H], W2t [C,H], b2 [C]) into a flat buffer."""
    return (p[OFF_W1:OFF_B1].view(H, D), p[OFF_B1:OFF_W2], p[OFF_W2:OFF_B2].view(C, H),
            p[OFF_B2:NPARAM])


class StepWorkspace:
    """Device scratch of the fused step for batch size ``B`` (zeroed once:
    the padding rows/columns the kernels never write must stay zero)."""

    def __init__(self, B, device, stats_ring=4096):
        if not 1 <= B <= MAX_BATCH:
            raise ValueError("fused MLP step supports 1 <= batch <= %d" % MAX_BATCH)
        self.B = B
        self.device = torch.device(device)
        n = hip().mlp_workspace_floats(B) if self.device.type == "cuda" else 1
        self.buf = torch.zeros(int(n), device=device, dtype=torch.float32)
        # global_step (advanced on the device by mlp_wgrad)
        self.ctr = torch.zeros(1, device=device, dtype=torch.int32)
        self.stats_ring = stats_ring
        self.stats = torch.zeros(stats_ring, 2, device=device, dtype=torch.float32)

    def global_step(self) -> int:
        return int(self.ctr[0].item())

    def set_global_step(self, s: int):
        self.ctr.fill_(int(s))


def _check(x, labels, B):
    if x.dtype != torch.float32 or not x.is_contiguous() or x.numel() != B * D or not x.is_cuda:
        raise ValueError("x must be a contiguous f32 GPU batch of B*784 values")
    if x.data_ptr() % 16:
        raise ValueError("x batch must be 16-byte aligned")
    if labels is not None and (labels.dtype != torch.int32 or labels.numel() != B
                               or not labels.is_contiguous()):
        raise ValueError("labels must be a contiguous int32 batch of B values")


def _check_flat(*ts):
    for t in ts:
        if t is not None and (t.numel() != NPARAM or t.dtype != torch.float32 or not t.is_cuda
                              or not t.is_contiguous()):
            raise ValueError("parameter/gradient buffers must be contiguous f32 [79510] on the GPU")


def step_direct(p, x, labels, ws: StepWorkspace, lr, stats=True):
    """One full SGD step in place on ``p`` for the batch (x [B,784], labels [B])."""
    _check(x, labels, ws.B)
    _check_flat(p)
    h, s = hip(), stream_handle()
    h.mlp_fwd(ptr(p), 0, 0.0, 0, ptr(x), ptr(ws.buf), ws.B, s)
    h.mlp_head(ptr(p), 0, 0.0, 0, ptr(labels), ptr(ws.buf), ws.B, s)
    h.mlp_wgrad(ptr(p), float(lr), 0, ptr(x), ptr(ws.buf), ptr(ws.ctr),
                ptr(ws.stats) if stats else 0, ws.stats_ring, ws.B, s)


def step_pipelined(p_old, p_new, x_prev, x, labels, ws: StepWorkspace, lr, apply, stats=True):
    """Two-launch single-GPU step: ``mlp_fwdapply`` applies the PREVIOUS step's SGD update
    (from the factors dz1/h/dlogits the last head left in ``ws`` and the previous batch
    ``x_prev``; W1 never materialises a gradient) reading ``p_old`` and writing ``p_new``,
    and runs this step's forward on the updated W1; ``mlp_head2`` (28 partial z1 slabs:
    the single-GPU K slicing, ``hip().mlp_single_ks()``) finishes the step.  ``apply=False`` (nothing pending): a plain copy + forward.  The
    last step's update stays pending until ``flush_pipelined``."""
    _check(x, labels, ws.B)
    _check(x_prev, None, ws.B)
    _check_flat(p_old, p_new)
    if p_old.data_ptr() == p_new.data_ptr():
        raise ValueError("the pipelined step needs distinct ping-pong buffers")
    h, s = hip(), stream_handle()
    h.mlp_fwdapply(ptr(p_old), ptr(p_new), float(lr) if apply else 0.0,
                   ptr(x_prev if apply else x), ptr(x), ptr(ws.buf), ptr(ws.ctr),
                   ptr(ws.stats) if stats else 0, ws.stats_ring, ws.B, 1 if apply else 0, s)
    h.mlp_head2(ptr(p_new), ptr(labels), ptr(ws.buf), ws.B, s)


def flush_pipelined(p_old, p_new, x_prev, ws: StepWorkspace, lr, stats=True):
    """Apply the pending update of the last pipelined step, ``p_old`` -> ``p_new`` (the
    ping-pong pair; the caller flips its parity): the apply half of ``mlp_fwdapply`` alone
    (same factors, same batch, same K slicing), with the step's stats record."""
    _check(x_prev, None, ws.B)
    _check_flat(p_old)
    _check_flat(p_new)
    hip().mlp_apply(ptr(p_old), ptr(p_new), float(lr), ptr(x_prev), ptr(ws.buf), ptr(ws.ctr),
                    ptr(ws.stats) if stats else 0, ws.stats_ring, ws.B, stream_handle())


def step_xgmi(p, x, labels, ws: StepWorkspace, lr, comm, stats=True):
    """One synchronous data-parallel SGD step in place on ``p`` with the gradient exchange
    fused into the weight-gradient kernel (``comm``: an ``XgmiComm`` with protocol "push";
    ``lr`` already divided by the world size).  Three launches, like ``step_direct``."""
    _check(x, labels, ws.B)
    _check_flat(p)
    h, s = hip(), stream_handle()
    h.mlp_fwd(ptr(p), 0, 0.0, 0, ptr(x), ptr(ws.buf), ws.B, s)
    h.mlp_head(ptr(p), 0, 0.0, 0, ptr(labels), ptr(ws.buf), ws.B, s)
    comm.mlp_wgrad(p, lr, x, ws, stats)


def step_xgmi_pipelined(p_old, p_new, x_prev, x, labels, ws: StepWorkspace, lr, apply, comm,
                        stats=True):
    """Two-launch data-parallel step of the fused engine: (1) step t-1's local gradient
    tiles exchanged over xGMI and applied (``p_old`` -> ``p_new``) inside the launch that
    runs step t's forward; (2) the plain head.  ``lr`` already divided by the world size;
    ``apply=False``: exchange of nothing useful + copy + forward.  The last update stays
    pending until ``flush_xgmi`` (which must run the same kernel: the exchange-epoch slots
    of a communicator belong to one kernel's tiling)."""
    _check(x, labels, ws.B)
    _check(x_prev, None, ws.B)
    _check_flat(p_old, p_new)
    if p_old.data_ptr() == p_new.data_ptr():
        raise ValueError("the pipelined step needs distinct ping-pong buffers")
    comm.mlp_fwdapply(p_old, p_new, lr, x_prev, x, ws, apply, stats)
    hip().mlp_head2(ptr(p_new), ptr(labels), ptr(ws.buf), ws.B, stream_handle(), XG_SLABS)


def flush_xgmi(p_old, p_new, x_prev, ws: StepWorkspace, lr, comm, stats=True):
    """Apply the pending update of the last pipelined fused step: the first launch once
    more (its forward on ``x_prev`` is discarded).  Result in ``p_new``."""
    _check(x_prev, None, ws.B)
    _check_flat(p_old, p_new)
    comm.mlp_fwdapply(p_old, p_new, lr, x_prev, x_prev, ws, True, stats)


def factor_plane(B):
    """Elements of one rank's dz1 plane in the factor engine's gather buffer ([BP][112], row-major)."""
    return HP * ((B + 15) // 16) * 16


def step_factor(p, x, labels, ws: StepWorkspace, lr, comm, dz1A, xstride, stats=True):
    """One synchronous data-parallel SGD step by sufficient-factor exchange (``comm``: an
    ``XgmiComm`` with protocol "push"; ``lr`` already divided by the world size).

    The head launch all-gathers every rank's backprop factors dz1 [B, 100] into ``dz1A``
    (zero-initialised [world, 112, BP]); every rank holds every rank's batch (rank q's at
    ``x + (q - rank) * xstride`` elements), so the weight-gradient launch forms the GLOBAL
    dW1 = sum_q dz1_q^T x_q locally and applies it -- 40 KB of factors per rank cross xGMI
    instead of the 313 KB W1 gradient.  Three launches, like ``step_direct``."""
    _check(x, labels, ws.B)
    _check_flat(p)
    if dz1A.numel() < comm.world_size * factor_plane(ws.B) or dz1A.dtype != torch.float32:
        raise ValueError("dz1A must hold world * 112 * BP f32 values")
    h, s = hip(), stream_handle()
    h.mlp_fwd(ptr(p), 0, 0.0, 0, ptr(x), ptr(ws.buf), ws.B, s)
    comm.mlp_head(p, labels, ws, dz1A)
    comm.mlp_wgrad_factor(p, lr, x, xstride, dz1A, ws, stats)


def step_factor_pipelined(p_old, p_new, x_prev, x, labels, ws: StepWorkspace, lr, apply, comm,
                          dz1A, xstride, stats=True):
    """Two-launch data-parallel step of the factor engine: (1) step t-1's GLOBAL update --
    W1 from every rank's gathered dz1 and resident previous batch, dW2/db1/db2 exchanged --
    fused with step t's forward; (2) the head of step t, which all-gathers dz1 into
    ``dz1A``.  ``lr`` already divided by the world size; ``apply=False``: copy + forward.
    The last update stays pending until ``flush_factor``."""
    _check(x, labels, ws.B)
    _check(x_prev, None, ws.B)
    _check_flat(p_old, p_new)
    if ws.B > 128:
        raise ValueError("the pipelined factor step supports batch <= 128")
    if dz1A.numel() < comm.world_size * factor_plane(ws.B):
        raise ValueError("dz1A must hold world * 112 * BP f32 values")
    comm.mlp_fwdapply_factor(p_old, p_new, lr, x_prev, x, xstride, dz1A, ws, apply, stats)
    comm.mlp_head(p_new, labels, ws, dz1A, nslab=FACTOR_SLABS)


def flush_factor(p, x_prev, ws: StepWorkspace, lr, comm, dz1A, xstride, stats=True):
    """Apply the pending update of the last pipelined factor step in place (the 3-launch
    factor engine's weight-gradient launch on the same factors and batches)."""
    _check(x_prev, None, ws.B)
    _check_flat(p)
    comm.mlp_wgrad_factor(p, lr, x_prev, xstride, dz1A, ws, stats)


def step_grad(p_old, x, labels, ws: StepWorkspace, grad, prev_grad=None, lr=0.0, p_new=None,
              stats=True):
    """Forward/backward writing ``grad``; optionally first applies ``prev_grad``.

    With ``prev_grad`` the step computes on ``p_new = p_old - lr * prev_grad``
    (published into ``p_new`` by the kernels) -- the deferred apply of sync DP.
    Returns the parameter buffer the gradient belongs to.
    """
    _check(x, labels, ws.B)
    _check_flat(p_old, grad, prev_grad, p_new)
    if prev_grad is not None and (p_new is None or p_new.data_ptr() == p_old.data_ptr()):
        raise ValueError("apply needs a distinct p_new buffer (ping-pong)")
    h, s = hip(), stream_handle()
    pg = ptr(prev_grad)
    pn = ptr(p_new) if prev_grad is not None else 0
    h.mlp_fwd(ptr(p_old), pg, float(lr), pn, ptr(x), ptr(ws.buf), ws.B, s)
    h.mlp_head(ptr(p_old), pg, float(lr), pn, ptr(labels), ptr(ws.buf), ws.B, s)
    h.mlp_wgrad(0, 0.0, ptr(grad), ptr(x), ptr(ws.buf), ptr(ws.ctr),
                ptr(ws.stats) if stats else 0, ws.stats_ring, ws.B, s)
    return p_new if prev_grad is not None else p_old


def to_tf_layout(flat, out, record=None):
    """Flat kernel layout -> TF checkpoint layout (kernels [in, out]) as ONE concatenated buffer
    [W1 784x100 | b1 | W2 100x10 | b2] (same segment offsets), optionally followed by the
    floats of ``record`` (e.g. the step's loss / accuracy) -- one launch on the GPU."""
    extra = 0 if record is None else record.numel()
    if out.numel() < NPARAM + extra:
        raise ValueError("output too small")
    if flat.is_cuda:
        hip().mlp_tf_layout(ptr(flat), ptr(out), 1, ptr(record), extra, stream_handle())
        return out
    W1t, b1, W2t, b2 = unflatten(flat)
    out[OFF_W1:OFF_B1].view(D, H).copy_(W1t.t())
    out[OFF_B1:OFF_W2].copy_(b1)
    out[OFF_W2:OFF_B2].view(H, C).copy_(W2t.t())
    out[OFF_B2:NPARAM].copy_(b2)
    if extra:
        out[NPARAM:NPARAM + extra].copy_(record.reshape(-1))
    return out


def from_tf_layout(tf, flat):
    """Inverse of ``to_tf_layout`` (the first NPARAM floats of ``tf``)."""
    if flat.is_cuda:
        hip().mlp_tf_layout(ptr(tf), ptr(flat), 0, 0, 0, stream_handle())
        return flat
    W1t, b1, W2t, b2 = unflatten(flat)
    W1t.copy_(tf[OFF_W1:OFF_B1].view(D, H).t())
    b1.copy_(tf[OFF_B1:OFF_W2])
    W2t.copy_(tf[OFF_W2:OFF_B2].view(H, C).t())
    b2.copy_(tf[OFF_B2:NPARAM])
    return flat


def reference_forward(p, x):
    W1t, b1, W2t, b2 = unflatten(p)
    h = torch.sigmoid(x @ W1t.t() + b1)
    return h, h @ W2t.t() + b2


def reference_step(p, x, labels):
    """Plain-torch forward/backward of worker.py's graph: (grad, loss, accuracy)."""
    W1t, b1, W2t, b2 = unflatten(p)
    B = x.shape[0]
    h, logits = reference_forward(p, x)
    lse = torch.logsumexp(logits, 1)
    lab = labels.long()
    loss = (lse - logits.gather(1, lab[:, None])[:, 0]).mean()
    acc = (logits.argmax(1) == lab).to(p.dtype).mean()
    prob = torch.softmax(logits, 1)
    dl = (prob - torch.nn.functional.one_hot(lab, C).to(p.dtype)) / B
    dz = (dl @ W2t) * h * (1 - h)
    g = torch.empty_like(p)
    gW1t, gb1, gW2t, gb2 = unflatten(g)
    gW1t.copy_(dz.t() @ x)
    gb1.copy_(dz.sum(0))
    gW2t.copy_(dl.t() @ h)
    gb2.copy_(dl.sum(0))
    return g, loss, acc
