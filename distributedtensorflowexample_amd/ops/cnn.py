"""CNN ops (ResNet-50 path) on the gfx950 kernels.

Convolutions are implicit GEMMs on the bf16 matrix cores
(``csrc/kernels/gemm_bf16.hip`` modes 1-3: the im2col / col2im gathers happen
in the glds staging, nothing is materialised); BatchNorm statistics are
fused into the forward convolution's epilogue; the rest lives in
``csrc/kernels/cnn.hip``.  Activations are NHWC bf16 tensors ``[N, H, W, C]``;
conv weights are ``[Cout, ldw]`` bf16 rows holding ``[KH][KW][Cin]`` (``ldw``
= KH*KW*Cin rounded up to 64, zero tail).  CPU tensors run f32 PyTorch
references of the same math.  North-star config 4 of BASELINE.json.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from ._ext import hip, ptr, stream_handle

# split-K partials through a workspace + reduce pass (DTFX_SPLITK_WS=0: f32 atomics into the output)
_SPLITK_WS = os.environ.get("DTFX_SPLITK_WS", "1") != "0"
# 1x1 / stride-1 convolutions with 64 / 128 / 256 reduction channels on the streaming kernels
# (csrc/kernels/conv1x1.hip); DTFX_CONV1X1=0: the implicit-GEMM path (A/B runs)
_CONV1X1 = os.environ.get("DTFX_CONV1X1", "1") != "0"


def _pointwise(KH, KW, stride, pad, M, K, N, w, stats, residual=None):
    """The streaming 1x1 kernels take this product: wide outputs (N >= 256, any epilogue) or
    the narrow reductions (N = 64 / 128: BN statistics required, no shortcut gradient)."""
    if not (_CONV1X1 and KH == 1 and KW == 1 and stride == 1 and pad == 0 and w.stride(0) % 8 == 0):
        return False
    if N < 256 and (not stats or residual is not None):
        return False
    return hip().conv1x1_applies(M, K, N)

BF16 = torch.bfloat16


def out_hw(H, W, k, stride, pad):
    return (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1


def kpad(kh, kw, c):
    return (kh * kw * c + 63) // 64 * 64


def _w4(w, Cout, KH, KW, C):
    """[Cout, ldw] row layout -> torch OIHW f32."""
    return w[:, :KH * KW * C].float().reshape(Cout, KH, KW, C).permute(0, 3, 1, 2)


def _nchw(x):
    return x.float().permute(0, 3, 1, 2)


def conv_fwd(x, w, KH, KW, stride, pad, colsum=None, colsq=None, residual=None):
    """y = conv(x, w) (NHWC bf16); optional fused BN statistics: the sum / sum of squares of y
    per output channel are ACCUMULATED into f32 ``colsum`` / ``colsq`` [Cout] (both or neither).

    GPU: the convolution epilogue writes per-tile partial rows (no same-address atomics) and
    ``colpart_reduce`` folds them into colsum / colsq."""
    N, H, W, C = x.shape
    Cout = w.shape[0]
    OH, OW = out_hw(H, W, KH, stride, pad)
    if not x.is_cuda:
        y = F.conv2d(_nchw(x), _w4(w, Cout, KH, KW, C), stride=stride, padding=pad)
        y = y.permute(0, 2, 3, 1)
        if residual is not None:
            y = y + residual.float()
        if colsum is not None:
            colsum += y.reshape(-1, Cout).sum(0)
        if colsq is not None:
            colsq += (y.reshape(-1, Cout) ** 2).sum(0)
        return y.to(BF16)
    y = torch.empty(N, OH, OW, Cout, device=x.device, dtype=BF16)
    if (colsum is not None and residual is None
            and hip().stem_conv_applies(H, W, C, Cout, KH, KW, stride, pad)):
        # the ResNet stem (7x7/2, 8 -> 64 channels): csrc/kernels/stem_conv.hip, input patch
        # staged once per 16 x 16 output tile; one partial statistics row per 64 pixels
        part = torch.empty(2, hip().stem_conv_fwd_rows(N, OH, OW), Cout, device=x.device)
        hip().stem_conv_fwd(N, H, W, ptr(x), ptr(w), w.stride(0), ptr(y), ptr(part[0]),
                            ptr(part[1]), stream_handle())
        hip().colpart_reduce(part.shape[1], Cout, ptr(part[0]), ptr(part[1]), ptr(colsum),
                             ptr(colsq), stream_handle())
        return y
    if (colsum is not None and residual is None
            and hip().conv3x3_c128_applies(H, W, C, Cout, KH, KW, stride, pad)):
        # layer2's 128-channel 3x3 conv: csrc/kernels/conv3x3_c128.hip (input patch staged
        # once per 4 x 28 output tile, weights streamed one tap at a time); 2 rows per tile
        part = torch.empty(2, 2 * (N * OH * OW // 112), Cout, device=x.device)
        hip().conv3x3_c128(1, N, H, W, ptr(x), ptr(w), w.stride(0), ptr(y), 0, 0, 0, 0, 0,
                           ptr(part[0]), ptr(part[1]), stream_handle())
        hip().colpart_reduce(part.shape[1], Cout, ptr(part[0]), ptr(part[1]), ptr(colsum),
                             ptr(colsq), stream_handle())
        return y
    if (colsum is not None and residual is None
            and hip().conv3x3_c64_applies(H, W, C, Cout, KH, KW, stride, pad)):
        # layer1's 64-channel 3x3 conv: csrc/kernels/conv3x3_c64.hip (weights resident in
        # LDS, input patch staged once per 8 x 28 output tile); 4 partial rows per tile
        part = torch.empty(2, 4 * (N * OH * OW // 224), Cout, device=x.device)
        hip().conv3x3_c64_fwd(N, H, W, ptr(x), ptr(w), w.stride(0), ptr(y), ptr(part[0]),
                              ptr(part[1]), stream_handle())
        hip().colpart_reduce(part.shape[1], Cout, ptr(part[0]), ptr(part[1]), ptr(colsum),
                             ptr(colsq), stream_handle())
        return y
    if residual is None and _pointwise(KH, KW, stride, pad, N * H * W, C, Cout, w, colsum is not None):
        # the 1x1 expansions (64 -> 256 ... 256 -> 1024) and reductions (256 -> 64 / 128,
        # 512 -> 128): weights in registers, pixels streamed; one partial statistics row per
        # persistent pixel block
        M = N * H * W
        ps = pq = None
        if colsum is not None:
            part = torch.empty(2, hip().conv1x1_rows(1, M, C, Cout), Cout, device=x.device)
            ps, pq = part[0], part[1]
        hip().conv1x1(1, M, C, Cout, ptr(x), ptr(w), w.stride(0), ptr(y), 0, 0, 0, 0, 0, ptr(ps),
                      ptr(pq), 0, stream_handle())
        if colsum is not None:
            hip().colpart_reduce(ps.shape[0], Cout, ptr(ps), ptr(pq), ptr(colsum), ptr(colsq),
                                 stream_handle())
        return y
    ps = pq = None
    if colsum is not None:
        rows = (N * OH * OW + 63) // 64  # one partial row per 64-row output slab
        part = torch.empty(2, rows, Cout, device=x.device)
        ps, pq = part[0], part[1]
    # few output tiles over a deep K (layer4): split-K partials + an epilogue pass
    nws = hip().conv_splitk_ws_floats(1, N, H, W, C, Cout, KH, KW, stride, pad)
    ws = torch.empty(nws, device=x.device) if nws else None
    hip().conv_bf16(1, N, H, W, C, Cout, KH, KW, stride, pad, ptr(x), ptr(w), w.stride(0), ptr(y),
                    0.0, ptr(residual), ptr(ps), ptr(pq), 0, stream_handle(), ws=ptr(ws),
                    ws_floats=nws)
    if colsum is not None:
        hip().colpart_reduce(ps.shape[0], Cout, ptr(ps), ptr(pq), ptr(colsum), ptr(colsq),
                             stream_handle())
    return y


def conv_dgrad(dy, w, x_shape, KH, KW, stride, pad, residual=None, bn=None, wt=None):
    """dx = conv^T(dy, w) (+ residual), NHWC bf16.

    ``bn = (y, x, mean, rstd, sum_dy, sum_dyxh)``: the input of this conv is
    ``y = relu(batchnorm(x) [+ shortcut])`` and its backward's reductions are fused into the
    dgrad epilogue: the result is ``de = (dgrad + residual) * (y > 0)`` (the gradient at the
    BN output, which is also the shortcut's gradient), and ``sum_dy += sum(de)``,
    ``sum_dyxh += sum(de * xhat)`` per channel (f32 [C]; the zeroed dbeta / dgamma slots).
    Finish with :func:`bn_bwd_apply`."""
    N, H, W, C = x_shape
    Cout = w.shape[0]
    if not dy.is_cuda:
        dx = torch.nn.grad.conv2d_input((N, C, H, W), _w4(w, Cout, KH, KW, C), _nchw(dy),
                                        stride=stride, padding=pad).permute(0, 2, 3, 1)
        if residual is not None:
            dx = dx + residual.float()
        if bn is not None:
            y, x, mean, rstd, sdy, sdx = bn
            dx = dx * (y.float() > 0)
            de = dx.to(BF16).float().reshape(-1, C)
            xh = (x.float().reshape(-1, C) - mean) * rstd
            sdy += de.sum(0)
            sdx += (de * xh).sum(0)
        return dx.to(BF16)
    dx = torch.empty(N, H, W, C, device=dy.device, dtype=BF16)
    if residual is None and hip().conv3x3_c128_applies(H, W, C, Cout, KH, KW, stride, pad):
        # layer2's 128-channel 3x3 conv: csrc/kernels/conv3x3_c128.hip (flipped weights in a
        # workspace, dy patch staged once per 4 x 28 tile, BN backward in the epilogue)
        wf = torch.empty(C, 9 * Cout, device=dy.device, dtype=BF16)
        if bn is None:
            hip().conv3x3_c128(2, N, H, W, ptr(dy), ptr(w), w.stride(0), ptr(dx), ptr(wf), 0, 0,
                               0, 0, 0, 0, stream_handle())
            return dx
        y, x, mean, rstd, sdy, sdx = bn
        part = torch.empty(2, 8 * (N * H * W // 112), C, device=dy.device)
        hip().conv3x3_c128(2, N, H, W, ptr(dy), ptr(w), w.stride(0), ptr(dx), ptr(wf), ptr(y),
                           ptr(x), ptr(mean), ptr(rstd), ptr(part[0]), ptr(part[1]),
                           stream_handle())
        hip().colpart_reduce(part.shape[1], C, ptr(part[0]), ptr(part[1]), ptr(sdy), ptr(sdx),
                             stream_handle())
        return dx
    if residual is None and hip().conv3x3_c64_applies(H, W, C, Cout, KH, KW, stride, pad):
        # layer1's 64-channel 3x3 conv: csrc/kernels/conv3x3_c64.hip (dy patch staged once
        # per 8 x 28 tile, flipped weights (a workspace) resident in LDS, BN backward in the
        # epilogue)
        wf = torch.empty(C, 9 * Cout, device=dy.device, dtype=BF16)
        if bn is None:
            hip().conv3x3_c64_dgrad(N, H, W, ptr(dy), ptr(w), w.stride(0), ptr(dx), 0, 0, 0, 0,
                                    0, 0, ptr(wf), stream_handle())
            return dx
        y, x, mean, rstd, sdy, sdx = bn
        part = torch.empty(2, 8 * (N * H * W // 224), C, device=dy.device)
        hip().conv3x3_c64_dgrad(N, H, W, ptr(dy), ptr(w), w.stride(0), ptr(dx), ptr(y), ptr(x),
                                ptr(mean), ptr(rstd), ptr(part[0]), ptr(part[1]), ptr(wf),
                                stream_handle())
        hip().colpart_reduce(part.shape[1], C, ptr(part[0]), ptr(part[1]), ptr(sdy), ptr(sdx),
                             stream_handle())
        return dx
    if _pointwise(KH, KW, stride, pad, N * H * W, Cout, C, w, bn is not None, residual):
        # conv1's data gradient (64 / 128 / 256 -> 256 ... 1024 channels, + shortcut gradient)
        # and conv3's (256 / 512 -> 64 / 128): the streaming 1x1 kernels, ReLU mask and BN
        # reductions fused
        M = N * H * W
        # transposed weights: formed here, or (``wt`` given) already there -- ResNet50 forms
        # every 1x1 data gradient's copy in one batched launch per step (w passed as 0)
        wp = ptr(w)
        if wt is None:
            wt = torch.empty(C, Cout, device=dy.device, dtype=BF16)
        else:
            wp = 0
        if bn is None:
            hip().conv1x1(2, M, Cout, C, ptr(dy), wp, w.stride(0), ptr(dx), ptr(residual), 0,
                          0, 0, 0, 0, 0, ptr(wt), stream_handle())
            return dx
        y, x, mean, rstd, sdy, sdx = bn
        if y.shape != dx.shape or x.shape != dx.shape:
            raise ValueError("fused BN backward: y and x must have the dgrad output's shape")
        part = torch.empty(2, hip().conv1x1_rows(2, M, Cout, C), C, device=dy.device)
        hip().conv1x1(2, M, Cout, C, ptr(dy), wp, w.stride(0), ptr(dx), ptr(residual), ptr(y),
                      ptr(x), ptr(mean), ptr(rstd), ptr(part[0]), ptr(part[1]), ptr(wt),
                      stream_handle())
        hip().colpart_reduce(part.shape[1], C, ptr(part[0]), ptr(part[1]), ptr(sdy), ptr(sdx),
                             stream_handle())
        return dx
    nws = hip().conv_splitk_ws_floats(2, N, H, W, C, Cout, KH, KW, stride, pad)
    ws = torch.empty(nws, device=dy.device) if nws else None  # split-K partials (layer4)
    if bn is None:
        hip().conv_bf16(2, N, H, W, C, Cout, KH, KW, stride, pad, ptr(dy), ptr(w), w.stride(0),
                        ptr(dx), 0.0, ptr(residual), 0, 0, 0, stream_handle(), ws=ptr(ws),
                        ws_floats=nws)
        return dx
    y, x, mean, rstd, sdy, sdx = bn
    if y.shape != dx.shape or x.shape != dx.shape:
        raise ValueError("fused BN backward: y and x must have the dgrad output's shape")
    # one partial row per 64-row output slab of each stride x stride phase class (the
    # kernel sizes every class like the largest, ceil(H / s) x ceil(W / s) pixels)
    hc, wc = -(-H // stride), -(-W // stride)
    rows = stride * stride * ((N * hc * wc + 63) // 64)
    part = torch.empty(2, rows, C, device=dy.device)
    hip().conv_bf16(2, N, H, W, C, Cout, KH, KW, stride, pad, ptr(dy), ptr(w), w.stride(0),
                    ptr(dx), 0.0, ptr(residual), ptr(part[0]), ptr(part[1]), 0, stream_handle(),
                    relu_y=ptr(y), bn_x=ptr(x), bn_mean=ptr(mean), bn_rstd=ptr(rstd), ws=ptr(ws),
                    ws_floats=nws)
    hip().colpart_reduce(rows, C, ptr(part[0]), ptr(part[1]), ptr(sdy), ptr(sdx), stream_handle())
    return dx


def bn_bwd_apply(de, x, mean, rstd, gamma, sum_dy, sum_dyxh):
    """dx of BatchNorm from the gradient at its output ``de`` and the final reductions
    (``conv_dgrad(..., bn=...)``): dx = gamma*rstd*(de - mean(de) - xhat*mean(de*xhat))."""
    C = x.shape[-1]
    M = x.numel() // C
    if not x.is_cuda:
        d = de.float().reshape(M, C)
        xh = (x.float().reshape(M, C) - mean) * rstd
        dx = gamma * rstd * (d - sum_dy / M - xh * sum_dyxh / M)
        return dx.reshape(x.shape).to(BF16)
    dx = torch.empty_like(x)
    hip().bn_bwd_apply(M, C, ptr(de), ptr(x), ptr(mean), ptr(rstd), ptr(gamma), ptr(sum_dy),
                       ptr(sum_dyxh), ptr(dx), stream_handle())
    return dx


def bn_prologue_applies(x, K, N, mode):
    """True when a 1x1 / stride-1 product over ``x``'s pixels reducing K channels to N runs on
    a 1x1 kernel with the BatchNorm prologue: mode 1 :func:`bn_out_conv1x1` (K = the block
    output's channels, N = the next conv's), mode 2 :func:`bn_in_conv1x1_dgrad` (K = the conv's
    output channels, N = its input channels), mode 3 :func:`bn_relu_conv1x1`.
    ``DTFX_BN_PROLOGUE=0`` keeps the separate passes (A/B runs); the wide-kernel variants
    (mode 3, and mode 2 on a non-narrow shape) follow ``DTFX_BN_PROLOGUE_WIDE``."""
    if not (x.is_cuda and _CONV1X1 and _BN_PRO):
        return False
    M = x.numel() // x.shape[-1]
    if not hip().conv1x1_pro_applies(mode, M, K, N):
        return False
    narrow = bool(hip().conv1x1_pro_applies(1, M, K, N))
    return narrow or _BN_PRO_WIDE


_BN_PRO = os.environ.get("DTFX_BN_PROLOGUE", "1") != "0"
# The prologue kernels form the BatchNorm coefficients themselves from the BN's sums / affine
# (bn_common.h BnCoefSrc; block 0 writes mean / rstd / running statistics) instead of reading
# the rows of a separate bn_fwd_coef / bn_bwd_coef launch.  DTFX_BN_COEF_FUSED=0: the separate
# launch (A/B runs).
_BN_COEF_FUSED = os.environ.get("DTFX_BN_COEF_FUSED", "1") != "0"
_BN_PRO_WIDE = os.environ.get("DTFX_BN_PROLOGUE_WIDE", "1") != "0"


def bn_out_conv1x1(c, s, q, M, gamma, beta, residual, w, colsum, colsq, eps=1e-5, run_mean=None,
                   run_var=None, momentum=0.9, res_bn=None):
    """A bottleneck's output and the next 1x1 conv in one pass over the conv3 output.

    ``out = relu(bn(c) + shortcut)`` (training-mode BatchNorm of ``c`` from its column sums
    ``s`` / ``q`` over ``M`` rows; shortcut = ``residual``, or -- ``res_bn = (s2, q2, gamma2,
    beta2, run_mean2, run_var2)`` -- ``residual`` normalised by its own BatchNorm), then
    ``y = out W^T`` (1x1, stride 1) with y's BatchNorm statistics accumulated into
    ``colsum`` / ``colsq``.  GPU: ``bn_fwd_coef`` + the narrow 1x1 kernel's prologue
    (csrc/kernels/conv1x1.hip, PRO 1), which writes ``out`` as it forms the product's operand --
    the separate ``bn_apply`` pass and the conv's read of its result become one pass.
    Returns (out, y, mean, rstd) or, with ``res_bn``, (out, y, mean, rstd, mean2, rstd2)."""
    if not c.is_cuda:
        r = bn_apply_stats(c, s, q, M, gamma, beta, residual, True, eps, run_mean, run_var,
                           momentum, res_bn=res_bn)
        y = conv_fwd(r[0], w, 1, 1, 1, 0, colsum=colsum, colsq=colsq)
        return (r[0], y) + tuple(r[1:])
    K = c.shape[-1]
    Nout = w.shape[0]
    Mrows = c.numel() // K
    dev = c.device
    st = torch.empty(4 if res_bn is not None else 2, K, device=dev)
    coef = torch.empty(4, K, device=dev)
    s2 = q2 = g2 = b2 = rm2 = rv2 = None
    if res_bn is not None:
        s2, q2, g2, b2, rm2, rv2 = res_bn
    out = torch.empty_like(c)
    y = torch.empty(*c.shape[:-1], Nout, device=dev, dtype=BF16)
    part = torch.empty(2, hip().conv1x1_rows(1, Mrows, K, Nout), Nout, device=dev)
    m2 = ptr(st[2] if res_bn is not None else None)
    r2 = ptr(st[3] if res_bn is not None else None)
    if _BN_COEF_FUSED:
        hip().conv1x1_pro_fwdbn(1, Mrows, K, Nout, ptr(c), ptr(residual), int(M), ptr(s), ptr(q),
                                float(eps), ptr(st[0]), ptr(st[1]), ptr(run_mean), ptr(run_var),
                                float(momentum), ptr(gamma), ptr(beta), ptr(s2), ptr(q2),
                                ptr(g2), ptr(b2), m2, r2, ptr(rm2), ptr(rv2), ptr(out), ptr(w),
                                w.stride(0), ptr(y), ptr(part[0]), ptr(part[1]), stream_handle())
    else:
        hip().bn_fwd_coef(int(M), K, ptr(s), ptr(q), float(eps), ptr(st[0]), ptr(st[1]),
                          ptr(run_mean), ptr(run_var), float(momentum), ptr(gamma), ptr(beta),
                          ptr(s2), ptr(q2), ptr(g2), ptr(b2), m2, r2, ptr(rm2), ptr(rv2),
                          ptr(coef), stream_handle())
        hip().conv1x1_pro(1, Mrows, K, Nout, ptr(c), ptr(residual), ptr(coef), ptr(out), ptr(w),
                          w.stride(0), ptr(y), 0, 0, 0, 0, 0, ptr(part[0]), ptr(part[1]), 0,
                          stream_handle())
    hip().colpart_reduce(part.shape[1], Nout, ptr(part[0]), ptr(part[1]), ptr(colsum), ptr(colsq),
                         stream_handle())
    if res_bn is None:
        return out, y, st[0], st[1]
    return out, y, st[0], st[1], st[2], st[3]


def bn_relu_conv1x1(c, s, q, M, gamma, beta, w, colsum, colsq, eps=1e-5, run_mean=None,
                    run_var=None, momentum=0.9):
    """``a = relu(bn(c))`` (training-mode BatchNorm from c's column sums) and the 1x1 / stride-1
    expansion conv ``y = a W^T`` in one pass over ``c``: the wide 1x1 kernel's prologue (PRO 3)
    forms ``a`` in LDS, writes it once (the backward reads it) and feeds it to the MFMAs -- the
    bn_apply pass and the conv's read of its result become one.  y's BatchNorm statistics are
    accumulated into ``colsum`` / ``colsq``.  Returns (a, y, mean, rstd)."""
    if not c.is_cuda:
        a, mean, rstd = bn_apply_stats(c, s, q, M, gamma, beta, None, True, eps, run_mean, run_var,
                                       momentum)
        return a, conv_fwd(a, w, 1, 1, 1, 0, colsum=colsum, colsq=colsq), mean, rstd
    K = c.shape[-1]
    Nout = w.shape[0]
    Mrows = c.numel() // K
    st = torch.empty(2, K, device=c.device)
    a = torch.empty_like(c)
    y = torch.empty(*c.shape[:-1], Nout, device=c.device, dtype=BF16)
    part = torch.empty(2, hip().conv1x1_rows(1, Mrows, K, Nout), Nout, device=c.device)
    if _BN_COEF_FUSED:
        hip().conv1x1_pro_fwdbn(3, Mrows, K, Nout, ptr(c), 0, int(M), ptr(s), ptr(q), float(eps),
                                ptr(st[0]), ptr(st[1]), ptr(run_mean), ptr(run_var),
                                float(momentum), ptr(gamma), ptr(beta), 0, 0, 0, 0, 0, 0, 0, 0,
                                ptr(a), ptr(w), w.stride(0), ptr(y), ptr(part[0]), ptr(part[1]),
                                stream_handle())
    else:
        coef = torch.empty(4, K, device=c.device)
        hip().bn_fwd_coef(int(M), K, ptr(s), ptr(q), float(eps), ptr(st[0]), ptr(st[1]),
                          ptr(run_mean), ptr(run_var), float(momentum), ptr(gamma), ptr(beta), 0,
                          0, 0, 0, 0, 0, 0, 0, ptr(coef), stream_handle())
        hip().conv1x1_pro(3, Mrows, K, Nout, ptr(c), 0, ptr(coef), ptr(a), ptr(w), w.stride(0),
                          ptr(y), 0, 0, 0, 0, 0, ptr(part[0]), ptr(part[1]), 0, stream_handle())
    hip().colpart_reduce(part.shape[1], Nout, ptr(part[0]), ptr(part[1]), ptr(colsum), ptr(colsq),
                         stream_handle())
    return a, y, st[0], st[1]


def bn_relu_conv3x3_applies(c, w):
    """The 64-channel 3x3 kernel (with its BatchNorm + ReLU prologue) takes ``conv(relu(bn(c)))``
    for these shapes.  Opt-in (``DTFX_BN_PROLOGUE_C64=1``): in the ResNet-50 step it measured
    11,742-11,752 vs 11,753-11,769 img/s for the separate bn_apply pass (interleaved, one box,
    ``profiles/r4/resnet_c64pro/``) -- the transform and the scattered writes of ``a`` sit in the
    kernel's staging phase, which the 64-channel forward cannot hide."""
    N, H, W, C = c.shape
    return (c.is_cuda and _BN_PRO and _BN_PRO_C64 and w.shape[0] == C
            and bool(hip().conv3x3_c64_applies(H, W, C, C, 3, 3, 1, 1)))


_BN_PRO_C64 = os.environ.get("DTFX_BN_PROLOGUE_C64", "0") == "1"


def bn_relu_conv3x3(c, s, q, M, gamma, beta, w, colsum, colsq, eps=1e-5, run_mean=None,
                    run_var=None, momentum=0.9):
    """``a = relu(bn(c))`` (training-mode BatchNorm from c's column sums) and the 3x3 / stride-1
    / pad-1 conv ``y = conv(a, w)`` with y's BatchNorm statistics accumulated into ``colsum`` /
    ``colsq``, in one pass over ``c`` (GPU: ``conv3x3_c64.hip``'s prologue forms ``a`` as the
    input patch is staged and writes each tile's own pixels of it once).  Returns
    (a, y, mean, rstd)."""
    if not c.is_cuda:
        a, mean, rstd = bn_apply_stats(c, s, q, M, gamma, beta, None, True, eps, run_mean, run_var,
                                       momentum)
        return a, conv_fwd(a, w, 3, 3, 1, 1, colsum=colsum, colsq=colsq), mean, rstd
    N, H, W, K = c.shape
    Cout = w.shape[0]
    st = torch.empty(2, K, device=c.device)
    coef = torch.empty(4, K, device=c.device)
    hip().bn_fwd_coef(int(M), K, ptr(s), ptr(q), float(eps), ptr(st[0]), ptr(st[1]), ptr(run_mean),
                      ptr(run_var), float(momentum), ptr(gamma), ptr(beta), 0, 0, 0, 0, 0, 0, 0, 0,
                      ptr(coef), stream_handle())
    a = torch.empty_like(c)
    y = torch.empty(N, H, W, Cout, device=c.device, dtype=BF16)
    part = torch.empty(2, 4 * (N * H * W // 224), Cout, device=c.device)
    hip().conv3x3_c64_fwd(N, H, W, ptr(c), ptr(w), w.stride(0), ptr(y), ptr(part[0]),
                          ptr(part[1]), stream_handle(), coef=ptr(coef), xo=ptr(a))
    hip().colpart_reduce(part.shape[1], Cout, ptr(part[0]), ptr(part[1]), ptr(colsum), ptr(colsq),
                         stream_handle())
    return a, y, st[0], st[1]


def bn_in_conv1x1_dgrad(de, c, mean, rstd, gamma, sum_dy, sum_dyxh, w, bn=None, want_dc=True,
                        residual=None, residual_s2=False, wt=None):
    """BatchNorm backward's apply half and the data gradient of the 1x1 conv that produced the
    BatchNorm's input, in one pass.

    ``de`` = dL/d(BN output) with the final reductions ``sum_dy`` / ``sum_dyxh`` (see
    :func:`conv_dgrad`'s ``bn``), ``c`` = the BN input (this conv's output): the conv's output
    gradient ``dc = bn_bwd_apply(de, c, ...)`` is formed inside the 1x1 dgrad kernel's prologue
    (PRO 2) and written out when ``want_dc`` (the weight gradient reads it); the product is
    ``conv_dgrad(dc, w, residual=residual, bn=bn)`` -- with ``bn = (y, x, mean, rstd, sum_dy,
    sum_dyxh)`` the fused BatchNorm backward of the conv's own input (optional: without it
    the narrow kernels run the plain data gradient, PRO 4).  ``residual_s2`` (wide kernels): the
    residual is a stride-2 1x1 conv's data gradient stored compact, ``[N, H / 2, W / 2, Cin]``
    (zero at odd rows / columns of the full grid -- never materialised).  Returns (dx, dc)."""
    if residual is not None and residual_s2:
        N_, H_, W_, _ = c.shape
        if tuple(residual.shape) != (N_, H_ // 2, W_ // 2, w.shape[1]) or H_ % 2 or W_ % 2:
            raise ValueError("residual_s2: residual must be [N, H/2, W/2, Cin] of an even grid")
    if not de.is_cuda:
        if residual is not None and residual_s2:
            full = torch.zeros(*c.shape[:-1], w.shape[1], dtype=residual.dtype)
            full[:, ::2, ::2] = residual
            residual = full
        dc = bn_bwd_apply(de, c, mean, rstd, gamma, sum_dy, sum_dyxh)
        N, H, W, _ = c.shape
        dx = conv_dgrad(dc, w, (N, H, W, w.shape[1]), 1, 1, 1, 0, residual=residual, bn=bn)
        return dx, dc
    K = c.shape[-1]          # the conv's output channels (the BN's)
    Cin = w.shape[1]
    M = c.numel() // K
    dev = c.device
    coef = None
    if not _BN_COEF_FUSED:
        coef = torch.empty(4, K, device=dev)
        hip().bn_bwd_coef(M, K, ptr(mean), ptr(rstd), ptr(gamma), ptr(sum_dy), ptr(sum_dyxh),
                          ptr(coef), stream_handle())
    dc = torch.empty_like(c) if want_dc else None
    dx = torch.empty(*c.shape[:-1], Cin, device=dev, dtype=BF16)
    wp = ptr(w)  # (wt given: the transposed copy is already there, see conv_dgrad)
    if wt is None:
        wt = torch.empty(Cin, K, device=dev, dtype=BF16)
    else:
        wp = 0
    y = x = bmean = brstd = sdy = sdx = part = None
    if bn is not None:
        y, x, bmean, brstd, sdy, sdx = bn
        if y.shape != dx.shape or x.shape != dx.shape:
            raise ValueError("fused BN backward: y and x must have the dgrad output's shape")
        part = torch.empty(2, hip().conv1x1_rows(2, M, K, Cin), Cin, device=dev)
    rh, rw = (c.shape[1], c.shape[2]) if residual is not None and residual_s2 else (0, 0)
    if coef is None:
        hip().conv1x1_pro_bwdbn(M, K, Cin, ptr(de), ptr(c), M, ptr(mean), ptr(rstd), ptr(gamma),
                                ptr(sum_dy), ptr(sum_dyxh), ptr(dc), wp, w.stride(0),
                                ptr(dx), ptr(residual), ptr(y), ptr(x), ptr(bmean), ptr(brstd),
                                ptr(None if part is None else part[0]),
                                ptr(None if part is None else part[1]), ptr(wt),
                                stream_handle(), res_h=rh, res_w=rw)
    else:
        hip().conv1x1_pro(2, M, K, Cin, ptr(de), ptr(c), ptr(coef), ptr(dc), wp, w.stride(0),
                          ptr(dx), ptr(residual), ptr(y), ptr(x), ptr(bmean), ptr(brstd),
                          ptr(None if part is None else part[0]),
                          ptr(None if part is None else part[1]), ptr(wt), stream_handle(),
                          res_h=rh, res_w=rw)
    if part is not None:
        hip().colpart_reduce(part.shape[1], Cin, ptr(part[0]), ptr(part[1]), ptr(sdy), ptr(sdx),
                             stream_handle())
    return dx, dc


def stem_wgrad_bn_applies(x, Cout, k, stride, pad):
    """The stem weight-gradient kernel (with its BatchNorm prologue) takes this conv of x
    (``DTFX_STEM_WGRAD_BN=0``: the separate apply pass, A/B runs)."""
    N, H, W, C = x.shape
    return (x.is_cuda and _STEM_WGRAD_BN
            and bool(hip().stem_conv_applies(H, W, C, Cout, k, k, stride, pad)))


_STEM_WGRAD_BN = os.environ.get("DTFX_STEM_WGRAD_BN", "1") != "0"


def wgrad_fold_planes(x_shape, Cout, KH, KW, stride, pad, ldw):
    """How many f32 split-K planes conv_wgrad of this shape leaves behind with ``planes``
    (0: the shape does not take the workspace path, or ``ldw`` pads the rows -- then it cannot
    be folded into the optimizer)."""
    N, H, W, C = x_shape
    if (not _SPLITK_WS or ldw != KH * KW * C or hip().stem_conv_applies(H, W, C, Cout, KH, KW, stride, pad)
            or hip().conv3x3_c64_applies(H, W, C, Cout, KH, KW, stride, pad)):
        return 0
    return int(hip().conv_wgrad_ws_floats(N, H, W, C, Cout, KH, KW, stride, pad))


def conv_wgrad(dy, x, dw, KH, KW, stride, pad, beta=1.0, bn_in=None, planes=None):
    """dw[:, :KH*KW*C] (f32 [Cout, ldw]) (+)= dL/dW.

    ``planes`` (GPU, :func:`wgrad_fold_planes` floats): the split-K partial planes are left
    there and ``dw`` is not touched -- the optimizer sums them (``sgd_momentum_mixed`` with
    segments; one GPU only: an all-reduce needs the reduced gradient).

    ``bn_in = (c, bcoef)`` (the ResNet stem only, see :func:`maxpool_bn_bwd`): ``dy`` is the
    gradient at the BatchNorm output behind this conv and the conv output gradient is formed
    as the kernel stages it, ``dc = bn_bwd_apply(dy, c)`` with the coefficients ``bcoef``."""
    N, H, W, C = x.shape
    Cout = dy.shape[-1]
    if bn_in is not None:
        if not (dy.is_cuda and hip().stem_conv_applies(H, W, C, Cout, KH, KW, stride, pad)
                and beta in (0.0, 1.0)):
            raise ValueError("conv_wgrad: the BatchNorm prologue is the stem kernel's (GPU)")
        c, bcoef = bn_in
        hip().stem_conv_wgrad(N, H, W, ptr(x), ptr(dy), ptr(dw), dw.stride(0), float(beta),
                              stream_handle(), bnx=ptr(c), coef=ptr(bcoef))
        return dw
    if not dy.is_cuda:
        g = torch.nn.grad.conv2d_weight(_nchw(x), (Cout, C, KH, KW), _nchw(dy), stride=stride,
                                        padding=pad)
        g = g.permute(0, 2, 3, 1).reshape(Cout, -1)
        k = KH * KW * C
        dw[:, :k] = g + (beta * dw[:, :k] if beta else 0)
        return dw
    if hip().stem_conv_applies(H, W, C, Cout, KH, KW, stride, pad) and beta in (0.0, 1.0):
        # the ResNet stem: csrc/kernels/stem_conv.hip (dy tile + input patch staged once per
        # 8 x 16 output tile, per-block partial gradient summed in registers)
        hip().stem_conv_wgrad(N, H, W, ptr(x), ptr(dy), ptr(dw), dw.stride(0), float(beta),
                              stream_handle())
        return dw
    if hip().conv3x3_c64_applies(H, W, C, Cout, KH, KW, stride, pad) and beta in (0.0, 1.0):
        # layer1's 64-channel 3x3 conv: csrc/kernels/conv3x3_c64.hip (dy tile + input patch
        # staged once per 4 x 28 tile, per-block partial gradient summed in registers)
        hip().conv3x3_c64_wgrad(N, H, W, ptr(x), ptr(dy), ptr(dw), dw.stride(0), float(beta),
                                stream_handle())
        return dw
    if planes is not None:
        nws = planes.numel()
        hip().conv_bf16(3, N, H, W, C, Cout, KH, KW, stride, pad, ptr(dy), ptr(x), dw.stride(0),
                        ptr(dw), float(beta), 0, 0, 0, 0, stream_handle(), ws=ptr(planes),
                        ws_floats=nws, defer_reduce=True)
        return dw
    # split-K partials through a workspace + one reduce pass instead of f32 atomics
    nws = hip().conv_wgrad_ws_floats(N, H, W, C, Cout, KH, KW, stride, pad) if _SPLITK_WS else 0
    ws = torch.empty(nws, device=dy.device) if nws else None
    hip().conv_bf16(3, N, H, W, C, Cout, KH, KW, stride, pad, ptr(dy), ptr(x), dw.stride(0),
                    ptr(dw), float(beta), 0, 0, 0, 0, stream_handle(), ws=ptr(ws), ws_floats=nws)
    return dw


# ---------------------------------------------------------------- BatchNorm
def bn_finalize(s, q, M, eps=1e-5, run_mean=None, run_var=None, momentum=0.9):
    C = s.numel()
    if not s.is_cuda:
        mean = s / M
        var = (q / M - mean * mean).clamp_min(0)
        if run_mean is not None:
            run_mean.mul_(momentum).add_((1 - momentum) * mean)
            run_var.mul_(momentum).add_((1 - momentum) * var * (M / max(M - 1, 1)))
        return mean, torch.rsqrt(var + eps)
    mean = torch.empty(C, device=s.device)
    rstd = torch.empty(C, device=s.device)
    hip().bn_finalize(C, int(M), ptr(s), ptr(q), float(eps), ptr(mean), ptr(rstd), ptr(run_mean),
                      ptr(run_var), float(momentum), stream_handle())
    return mean, rstd


def bn_apply(x, mean, rstd, gamma, beta, residual=None, relu=True):
    C = x.shape[-1]
    if not x.is_cuda:
        y = (x.float() - mean) * rstd * gamma + beta
        if residual is not None:
            y = y + residual.float()
        if relu:
            y = torch.relu(y)
        return y.to(BF16)
    y = torch.empty_like(x)
    hip().bn_apply(x.numel() // C, C, ptr(x), ptr(mean), ptr(rstd), ptr(gamma), ptr(beta),
                   ptr(residual), int(relu), ptr(y), stream_handle())
    return y


def bn_apply_stats(x, s, q, M, gamma, beta, residual=None, relu=True, eps=1e-5, run_mean=None,
                   run_var=None, momentum=0.9, res_bn=None):
    """Training-mode forward BatchNorm from the conv epilogue's column sums ``s`` / ``q``
    (sum, sum of squares over ``M`` rows): ``bn_finalize`` + ``bn_apply`` in one launch on
    the GPU (mean / rstd formed per thread, block 0 stores them and updates the running
    statistics).  ``res_bn = (s2, q2, gamma2, beta2, run_mean2, run_var2)``: ``residual`` is
    a raw conv output normalised by its own statistics before the add (a bottleneck's
    downsample shortcut, never materialised).  Returns (y, mean, rstd) or, with ``res_bn``,
    (y, mean, rstd, mean2, rstd2)."""
    if not x.is_cuda:
        mean, rstd = bn_finalize(s, q, M, eps, run_mean, run_var, momentum)
        extra = ()
        if res_bn is not None:
            s2, q2, g2, b2, rm2, rv2 = res_bn
            m2, r2 = bn_finalize(s2, q2, M, eps, rm2, rv2, momentum)
            residual = bn_apply(residual, m2, r2, g2, b2, relu=False)
            extra = (m2, r2)
        return (bn_apply(x, mean, rstd, gamma, beta, residual, relu), mean, rstd) + extra
    C = x.shape[-1]
    mean = torch.empty(C, device=x.device)
    rstd = torch.empty(C, device=x.device)
    y = torch.empty_like(x)
    s2 = q2 = g2 = b2 = rm2 = rv2 = m2 = r2 = None
    if res_bn is not None:
        s2, q2, g2, b2, rm2, rv2 = res_bn
        m2 = torch.empty(C, device=x.device)
        r2 = torch.empty(C, device=x.device)
    hip().bn_apply_stats(x.numel() // C, C, ptr(x), ptr(s), ptr(q), float(eps), ptr(mean), ptr(rstd),
                         ptr(run_mean), ptr(run_var), float(momentum), ptr(gamma), ptr(beta),
                         ptr(residual), int(relu), ptr(y), ptr(s2), ptr(q2), ptr(g2), ptr(b2),
                         ptr(m2), ptr(r2), ptr(rm2), ptr(rv2), stream_handle())
    return (y, mean, rstd) if res_bn is None else (y, mean, rstd, m2, r2)


def bn_bwd(dy, y, x, mean, rstd, gamma, dgamma, dbeta, relu=True, want_dres=False,
           grads_zeroed=False, apply=True):
    """Backward of y = act(bn(x) [+ res]).  Accumulates dgamma/dbeta; returns (dx, dres)
    where dres = dy * act'(y) is the gradient of the residual input (if requested).
    ``apply=False`` (GPU, no ReLU): only the reductions -- the caller forms dx in a consumer's
    prologue (:func:`bn_in_conv1x1_dgrad`); returns (None, None).

    ``grads_zeroed=True`` (the model's per-step zeroed gradient slots) lets the GPU kernels
    reduce straight into dgamma / dbeta -- they are exactly sum(dy_eff * xhat) / sum(dy_eff)
    -- instead of into zeroed temporaries that are then added."""
    C = x.shape[-1]
    M = x.numel() // C
    if not x.is_cuda:
        de = dy.float() * (y.float() > 0) if relu else dy.float()
        de2 = de.reshape(M, C)
        xh = (x.float().reshape(M, C) - mean) * rstd
        sdy, sdx = de2.sum(0), (de2 * xh).sum(0)
        dx = gamma * rstd * (de2 - sdy / M - xh * sdx / M)
        dgamma += sdx
        dbeta += sdy
        return dx.reshape(x.shape).to(BF16), (de.to(BF16) if want_dres else None)
    if grads_zeroed:
        sdy, sdx = dbeta, dgamma
    else:
        sums = torch.zeros(2, C, device=x.device)
        sdy, sdx = sums[0], sums[1]
    if not apply and (relu or want_dres):
        raise ValueError("bn_bwd(apply=False): reductions of an un-masked gradient only")
    rows = hip().bn_bwd_scratch_rows(M, C)
    scratch = torch.empty(2 * rows * C, device=x.device)
    dx = torch.empty_like(x) if apply else None
    dres = torch.empty_like(x) if want_dres else None
    hip().bn_bwd(M, C, ptr(dy), ptr(y), ptr(x), ptr(mean), ptr(rstd), ptr(gamma), int(relu),
                 ptr(sdy), ptr(sdx), ptr(scratch), ptr(dx), ptr(dres), stream_handle())
    if not grads_zeroed:
        dgamma += sdx
        dbeta += sdy
    return dx, dres


# ---------------------------------------------------------------- pooling
def maxpool_fwd(x):
    """3x3 / stride 2 / pad 1 max pool; returns (y, argmax tap index uint8)."""
    N, H, W, C = x.shape
    OH, OW = out_hw(H, W, 3, 2, 1)
    if not x.is_cuda:
        xp = F.pad(_nchw(x), (1, 1, 1, 1), value=float("-inf"))
        cols = F.unfold(xp, 3, stride=2).view(N, C, 9, OH * OW)
        y, idx = cols.max(2)
        y = y.view(N, C, OH, OW).permute(0, 2, 3, 1).to(BF16)
        idx = idx.view(N, C, OH, OW).permute(0, 2, 3, 1).to(torch.uint8).contiguous()
        return y.contiguous(), idx
    y = torch.empty(N, OH, OW, C, device=x.device, dtype=BF16)
    idx = torch.empty(N, OH, OW, C, device=x.device, dtype=torch.uint8)
    hip().maxpool_fwd(N, H, W, C, ptr(x), ptr(y), ptr(idx), stream_handle())
    return y, idx


def bn_maxpool_fwd(c, s, q, M, gamma, beta, eps=1e-5, run_mean=None, run_var=None,
                   momentum=0.9):
    """The ResNet stem's ``maxpool(relu(bn(c)))`` (training-mode BatchNorm from c's column sums
    ``s`` / ``q`` over ``M`` rows) without materialising ``relu(bn(c))``.
    Returns (y, idx, mean, rstd, fcoef); ``fcoef`` (GPU: the [4][C] BatchNorm coefficients,
    CPU: None) goes to :func:`maxpool_bn_bwd`."""
    if not c.is_cuda:
        a, mean, rstd = bn_apply_stats(c, s, q, M, gamma, beta, None, True, eps, run_mean, run_var,
                                       momentum)
        y, idx = maxpool_fwd(a)
        return y, idx, mean, rstd, None
    N, H, W, C = c.shape
    OH, OW = out_hw(H, W, 3, 2, 1)
    st = torch.empty(2, C, device=c.device)
    fcoef = torch.empty(4, C, device=c.device)
    hip().bn_fwd_coef(int(M), C, ptr(s), ptr(q), float(eps), ptr(st[0]), ptr(st[1]), ptr(run_mean),
                      ptr(run_var), float(momentum), ptr(gamma), ptr(beta), 0, 0, 0, 0, 0, 0, 0, 0,
                      ptr(fcoef), stream_handle())
    y = torch.empty(N, OH, OW, C, device=c.device, dtype=BF16)
    idx = torch.empty(N, OH, OW, C, device=c.device, dtype=torch.uint8)
    hip().maxpool_bn_fwd(N, H, W, C, ptr(c), ptr(fcoef), ptr(y), ptr(idx), stream_handle())
    return y, idx, st[0], st[1], fcoef


def maxpool_bn_bwd(dy, idx, c, mean, rstd, gamma, beta, fcoef, dgamma, dbeta, apply=True):
    """Backward of :func:`bn_maxpool_fwd`: dL/dc from the pool's output gradient ``dy``;
    dgamma / dbeta are the (per-step zeroed) gradient slots, which receive BatchNorm backward's
    two sums.  GPU: one pass gathers the pool gradient, masks it with the ReLU recomputed from
    ``c``, reduces the sums and writes ``de``; the streaming apply reads ``de`` and ``c``
    (``relu(bn(c))`` is never read or written).  ``apply=False`` (GPU): return ``(de,
    bcoef)`` instead of dL/dc -- the stem weight gradient forms dL/dc itself
    (:func:`conv_wgrad` ``bn_in``)."""
    if not c.is_cuda:
        a = bn_apply(c, mean, rstd, gamma, beta, None, relu=True)
        da = maxpool_bwd(dy, idx, c.shape)
        dc, _ = bn_bwd(da, a, c, mean, rstd, gamma, dgamma, dbeta, relu=True, grads_zeroed=True)
        return dc
    N, H, W, C = c.shape
    rows = hip().maxpool_bn_bwd_rows(N, H, W, C)
    scratch = torch.empty(2 * rows * C, device=c.device)
    de = torch.empty_like(c)
    dc = torch.empty_like(c) if apply else None
    bcoef = None if apply else torch.empty(4, C, device=c.device)
    hip().maxpool_bn_bwd(N, H, W, C, ptr(dy), ptr(idx), ptr(c), ptr(fcoef), ptr(mean), ptr(rstd),
                         ptr(gamma), ptr(dbeta), ptr(dgamma), ptr(scratch), ptr(de), ptr(dc),
                         ptr(bcoef), stream_handle())
    return dc if apply else (de, bcoef)


def maxpool_bwd(dy, idx, x_shape):
    N, H, W, C = x_shape
    if not dy.is_cuda:
        OH, OW = dy.shape[1], dy.shape[2]
        g = torch.zeros(N, C, 9, OH * OW)
        g.scatter_(2, idx.permute(0, 3, 1, 2).reshape(N, C, 1, OH * OW).long(),
                   dy.float().permute(0, 3, 1, 2).reshape(N, C, 1, OH * OW))
        dx = F.fold(g.view(N, C * 9, OH * OW), (H + 2, W + 2), 3, stride=2)[:, :, 1:-1, 1:-1]
        return dx.permute(0, 2, 3, 1).contiguous().to(BF16)
    dx = torch.empty(N, H, W, C, device=dy.device, dtype=BF16)
    hip().maxpool_bwd(N, H, W, C, ptr(dy), ptr(idx), ptr(dx), stream_handle())
    return dx


def avgpool_fwd(x):
    N, H, W, C = x.shape
    if not x.is_cuda:
        return x.float().mean((1, 2)).to(BF16)
    y = torch.empty(N, C, device=x.device, dtype=BF16)
    hip().avgpool_fwd(N, H * W, C, ptr(x), ptr(y), stream_handle())
    return y


def avgpool_bwd(dy, x_shape):
    N, H, W, C = x_shape
    if not dy.is_cuda:
        return (dy.float()[:, None, None, :] / (H * W)).expand(N, H, W, C).contiguous().to(BF16)
    dx = torch.empty(N, H, W, C, device=dy.device, dtype=BF16)
    hip().avgpool_bwd(N, H * W, C, ptr(dy), ptr(dx), stream_handle())
    return dx


def sgd_momentum_mixed(p, g, v, pb, lr, momentum=0.9, wd=0.0, gscale=1.0, segs=None):
    """Momentum SGD on the f32 master (bf16 copy refreshed).  ``segs`` (GPU): int64 [n][5]
    table of ranges whose gradient is the sum of split-K planes (see conv_wgrad ``planes``)."""
    if segs is not None and p.is_cuda:
        hip().sgd_momentum_mixed(p.numel(), ptr(p), ptr(g), ptr(v), ptr(pb), float(lr),
                                 float(momentum), float(wd), float(gscale), stream_handle(),
                                 segs=ptr(segs), nseg=int(segs.shape[0]))
        return
    if not p.is_cuda:
        v.mul_(momentum).add_(g * gscale + wd * p)
        p.sub_(lr * v)
        if pb is not None:
            pb.copy_(p)
        return
    hip().sgd_momentum_mixed(p.numel(), ptr(p), ptr(g), ptr(v), ptr(pb), float(lr), float(momentum),
                             float(wd), float(gscale), stream_handle())
