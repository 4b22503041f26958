"""ResNet-50 (v1.5) image classifier on the bf16 gfx950 kernels.

North-star config 4 of BASELINE.json ("ResNet-50 synthetic ImageNet,
MirroredStrategy-style all-reduce on 8x MI355X"); the reference only has an
MNIST MLP (worker.py:47-54), so the architecture is the public ResNet-50 v1.5
(stride on the 3x3 conv of each down-sampling bottleneck).

MI355X-first design:

* NHWC bf16 activations; every convolution is an implicit GEMM on the bf16
  matrix cores (``ops.cnn.conv_*``: the im2col/col2im gathers run inside the
  GEMM's LDS staging) and the forward convolution's epilogue also produces
  the BatchNorm batch statistics (sum and sum of squares per channel), so BN
  costs one finalize + one fused apply(+residual +ReLU) pass;
* flat f32 master / bf16 working copy / f32 gradient / momentum buffers with
  64-element aligned slots; one all-reduce bucket per bottleneck block,
  released as soon as that block's backward finishes;
* the 3-channel input is stored with 8 channels (zero padded) so every
  gather moves 16-byte vectors; the 1000-way classifier is padded to 1024
  output rows (zero weights, masked in the loss).
"""
from __future__ import annotations

import math

import torch

from ..ops import bf16 as B16
from ..ops import cnn as CN
from ..ops import init as I
from ..ops import transformer as TR

BF16 = torch.bfloat16
ALIGN = 64
STAGES = [(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]  # (width, blocks, stride)
IN_CH = 8          # 3 image channels + 5 zero channels
NUM_CLASSES = 1000
CLS_PAD = 1024


def conv_specs(stages=STAGES, in_ch=IN_CH):
    """[(name, Cin, Cout, k, stride, pad)] in forward order."""
    L = [("conv1", in_ch, 64, 7, 2, 3)]
    cin = 64
    for si, (w, nb, st) in enumerate(stages):
        for b in range(nb):
            s = st if b == 0 else 1
            p = "layer%d.%d." % (si + 1, b)
            L += [(p + "conv1", cin, w, 1, 1, 0), (p + "conv2", w, w, 3, s, 1),
                  (p + "conv3", w, 4 * w, 1, 1, 0)]
            if b == 0:
                L.append((p + "downsample", cin, 4 * w, 1, s, 0))
            cin = 4 * w
    return L


class ResNetParams:
    def __init__(self, device, seed=0, stages=STAGES, num_classes=NUM_CLASSES):
        self.convs = conv_specs(stages)
        self.stages = stages
        self.num_classes = num_classes
        self.cls_pad = (num_classes + 63) // 64 * 64
        layout = []  # (name, shape, kind)
        for name, cin, cout, k, s, p in self.convs:
            layout.append((name + ".weight", (cout, CN.kpad(k, k, cin)), ("he", k * k * cin, k * k * cin)))
            layout.append((name + ".bn.gamma", (cout,), "ones"))
            layout.append((name + ".bn.beta", (cout,), "zeros"))
        feat = 4 * stages[-1][0]
        layout.append(("fc.weight", (self.cls_pad, feat), ("normal", 0.01)))
        layout.append(("fc.bias", (self.cls_pad,), "zeros"))
        self.layout = layout
        self.offsets = {}
        off = 0
        for name, shape, _ in layout:
            self.offsets[name] = (off, shape)
            off += (math.prod(shape) + ALIGN - 1) // ALIGN * ALIGN
        self.numel = off
        dev = torch.device(device)
        self.master = torch.zeros(off, device=dev)
        self.grad = torch.zeros(off, device=dev)
        self.mom = torch.zeros(off, device=dev)
        self.bf = torch.zeros(off, device=dev, dtype=BF16)
        for i, (name, shape, kind) in enumerate(layout):
            t = self.view(self.master, name)
            if isinstance(kind, tuple) and kind[0] == "he":
                k_real = kind[1]
                tmp = torch.empty(shape[0] * k_real, device=dev)
                I.fill_(tmp, "normal", 0.0, math.sqrt(2.0 / kind[2]), seed=seed, offset=i << 40)
                t[:, :k_real] = tmp.view(shape[0], k_real)
                if name == "conv1.weight":  # pad input channels 3..7 carry no weight
                    t[:, :k_real].view(shape[0], -1, IN_CH)[:, :, 3:] = 0
            elif isinstance(kind, tuple) and kind[0] == "normal":
                I.fill_(t.view(-1), "normal", 0.0, kind[1], seed=seed, offset=i << 40)
                t[num_classes:].zero_()
            elif kind == "ones":
                t.fill_(1.0)
        TR.cast_bf16(self.master, self.bf)
        # BatchNorm running statistics (not trained; checkpointed)
        self.running = {}
        for name, cin, cout, k, s, p in self.convs:
            self.running[name] = (torch.zeros(cout, device=dev), torch.ones(cout, device=dev))
        # one bucket per bottleneck block (+ stem, + head), as flat ranges in forward order
        starts = [0]
        for name, *_ in self.convs:
            if name.endswith(".conv1") and name != "conv1":
                starts.append(self.offsets[name + ".weight"][0])
        starts.append(self.offsets["fc.weight"][0])
        starts.append(off)
        self.buckets = [(starts[i], starts[i + 1]) for i in range(len(starts) - 1)]

    def view(self, flat, name):
        off, shape = self.offsets[name]
        return flat[off:off + math.prod(shape)].view(shape)

    def P(self, n):
        return self.view(self.master, n)

    def W(self, n):
        return self.view(self.bf, n)

    def G(self, n):
        return self.view(self.grad, n)


class ResNet50:
    """Explicit forward + backward over the HIP ops (training mode BatchNorm)."""

    def __init__(self, device, seed=0, stages=STAGES, num_classes=NUM_CLASSES, bn_eps=1e-5):
        self.device = torch.device(device)
        self.params = ResNetParams(device, seed, stages, num_classes)
        self.specs = {c[0]: c for c in self.params.convs}
        self.eps = bn_eps
        tot = sum(2 * c[2] for c in self.params.convs)
        self._stats_flat = torch.zeros(tot, device=self.device)
        self._stats, off = {}, 0
        for name, cin, cout, *_ in self.params.convs:
            self._stats[name] = (self._stats_flat[off:off + cout],
                                 self._stats_flat[off + cout:off + 2 * cout])
            off += 2 * cout
        # weight gradients on a second HIP stream (set by the trainer): each only needs its
        # conv's output gradient and saved input, so it overlaps the data-gradient / BatchNorm
        # chain.  ``wgrad_sync_buckets``: join before every gradient-bucket hook (sync DP).
        self.wgrad_stream = None
        self.wgrad_sync_buckets = True
        self._keep = []  # operands the side stream still reads

    # conv + fused BN statistics (column sums in the conv epilogue)
    def _conv_bn(self, name, x):
        _, cin, cout, k, s, p = self.specs[name]
        P = self.params
        cs, cq = self._stats[name]
        y = CN.conv_fwd(x, P.W(name + ".weight"), k, k, s, p, colsum=cs, colsq=cq)
        return y, (cs, cq, y.numel() // cout)

    # finalize (mean / rstd, running statistics) + apply (+ residual, ReLU) in one launch
    def _bn_apply(self, name, y, st, residual=None, relu=True, res_bn=None):
        P = self.params
        cs, cq, M = st
        rm, rv = P.running[name]
        return CN.bn_apply_stats(y, cs, cq, M, P.P(name + ".bn.gamma"), P.P(name + ".bn.beta"),
                                 residual, relu, self.eps, rm, rv, res_bn=res_bn)

    def forward_backward(self, images, labels, on_bucket_ready=None):
        """images: NHWC bf16 [N, H, W, 8]; labels int32 [N].  Returns (loss, accuracy)."""
        P = self.params
        N = images.shape[0]
        P.grad.zero_()
        self._stats_flat.zero_()  # every BN's (sum, sum of squares) accumulators, one memset
        saved = {}
        c, st = self._conv_bn("conv1", images)
        a, m, r = self._bn_apply("conv1", c, st)
        saved["conv1"] = (images, c, m, r, a)
        x, idx = CN.maxpool_fwd(a)
        blocks = []
        for si, (w, nb, st_) in enumerate(P.stages):
            for b in range(nb):
                pre = "layer%d.%d." % (si + 1, b)
                x_in = x
                c1, s1 = self._conv_bn(pre + "conv1", x_in)
                a1, m1, r1 = self._bn_apply(pre + "conv1", c1, s1)
                c2, s2 = self._conv_bn(pre + "conv2", a1)
                a2, m2, r2 = self._bn_apply(pre + "conv2", c2, s2)
                c3, s3 = self._conv_bn(pre + "conv3", a2)
                if b == 0:
                    # out = relu(bn3(c3) + bn_ds(downsample(x))) in one pass: the normalised
                    # shortcut is never materialised
                    cs_, sds = self._conv_bn(pre + "downsample", x_in)
                    rm, rv = P.running[pre + "downsample"]
                    nd = pre + "downsample.bn."
                    out, m3, r3, ms, rs = self._bn_apply(
                        pre + "conv3", c3, s3, residual=cs_, relu=True,
                        res_bn=(sds[0], sds[1], P.P(nd + "gamma"), P.P(nd + "beta"), rm, rv))
                    ds = (cs_, ms, rs)
                else:
                    ds = None
                    out, m3, r3 = self._bn_apply(pre + "conv3", c3, s3, residual=x_in, relu=True)
                blocks.append((pre, x_in, (c1, m1, r1, a1), (c2, m2, r2, a2), (c3, m3, r3), ds, out))
                x = out
        pooled = CN.avgpool_fwd(x)                               # [N, 2048]
        logits = B16.gemm(pooled, P.W("fc.weight"), False, True, bias=P.P("fc.bias"),
                          out_dtype=torch.float32)                # [N, 1024]
        loss_rows, correct, dlog = TR.mlm_xent(logits, labels, P.num_classes, 1.0 / N)
        loss = loss_rows.sum() / N
        acc = correct.sum() / N
        # ---------------- backward
        B16.gemm(dlog, pooled, True, False, out=P.G("fc.weight"), beta=1.0)
        B16.colsum(dlog, out=P.G("fc.bias"), beta=1.0)
        dpool = B16.gemm(dlog, P.W("fc.weight"))
        if on_bucket_ready is not None:
            on_bucket_ready(len(P.buckets) - 1)
        dx = CN.avgpool_bwd(dpool, x.shape)
        bucket = len(P.buckets) - 2
        ws = self.wgrad_stream
        dx_is_de = False  # dx already dL/d(BN output) of the block's conv3 (fused reductions)
        for i in range(len(blocks) - 1, -1, -1):
            pre, x_in, (c1, m1, r1, a1), (c2, m2, r2, a2), (c3, m3, r3), ds, out = blocks[i]
            # the previous block's conv3 BatchNorm consumes this block's input gradient:
            # its reductions go into this block's last dgrad epilogue
            prev = blocks[i - 1] if i > 0 else None
            fuse = None if prev is None else (prev[0] + "conv3", x_in, prev[4])
            dx = self._block_bwd(pre, dx, x_in, c1, m1, r1, a1, c2, m2, r2, a2, c3, m3, r3, ds,
                                 out, dout_is_de=dx_is_de, fuse_prev=fuse)
            dx_is_de = fuse is not None
            if on_bucket_ready is not None:
                if ws is not None and self.wgrad_sync_buckets:
                    torch.cuda.current_stream(dx.device).wait_stream(ws)
                on_bucket_ready(bucket)
            bucket -= 1
        da = CN.maxpool_bwd(dx, idx, saved["conv1"][4].shape)
        img, c, m, r, a = saved["conv1"]
        dc, _ = CN.bn_bwd(da, a, c, m, r, P.P("conv1.bn.gamma"), P.G("conv1.bn.gamma"),
                          P.G("conv1.bn.beta"), relu=True, grads_zeroed=True)
        _, cin, cout, k, s, p = self.specs["conv1"]
        CN.conv_wgrad(dc, img, P.G("conv1.weight"), k, k, s, p, beta=1.0)
        if ws is not None:  # join: every gradient final on the main stream
            torch.cuda.current_stream(dc.device).wait_stream(ws)
            self._keep.clear()
        if on_bucket_ready is not None:
            on_bucket_ready(0)
        return loss, acc

    def _bn_bwd(self, name, dy, y, x, mean, rstd, relu=True, want_dres=False):
        P = self.params
        return CN.bn_bwd(dy, y, x, mean, rstd, P.P(name + ".bn.gamma"), P.G(name + ".bn.gamma"),
                         P.G(name + ".bn.beta"), relu, want_dres, grads_zeroed=True)

    def _bn_fused(self, name, y, x, mean, rstd):
        """``bn`` argument of CN.conv_dgrad: BatchNorm ``name`` (input x, post-ReLU output y)
        has its backward reductions fused into the dgrad that produces its output gradient,
        straight into the (per-step zeroed) dbeta / dgamma slots."""
        P = self.params
        return (y, x, mean, rstd, P.G(name + ".bn.beta"), P.G(name + ".bn.gamma"))

    def _bn_apply_bwd(self, name, de, x, mean, rstd):
        P = self.params
        return CN.bn_bwd_apply(de, x, mean, rstd, P.P(name + ".bn.gamma"), P.G(name + ".bn.beta"),
                               P.G(name + ".bn.gamma"))

    def _wgrad_dgrad(self, name, dc, x_in, residual=None, need_dx=True, bn=None):
        P = self.params
        _, cin, cout, k, s, p = self.specs[name]
        ws = self.wgrad_stream
        if ws is None:
            CN.conv_wgrad(dc, x_in, P.G(name + ".weight"), k, k, s, p, beta=1.0)
        else:  # weight gradient beside the data gradient (operands kept alive until the join)
            ws.wait_stream(torch.cuda.current_stream(dc.device))
            with torch.cuda.stream(ws):
                CN.conv_wgrad(dc, x_in, P.G(name + ".weight"), k, k, s, p, beta=1.0)
            self._keep.append((dc, x_in))
        if not need_dx:
            return None
        return CN.conv_dgrad(dc, P.W(name + ".weight"), x_in.shape, k, k, s, p, residual=residual,
                             bn=bn)

    def _block_bwd(self, pre, dout, x_in, c1, m1, r1, a1, c2, m2, r2, a2, c3, m3, r3, ds, out,
                   dout_is_de=False, fuse_prev=None):
        """Backward of one bottleneck.  ``dout_is_de``: ``dout`` is already the gradient at
        conv3's BN output with its reductions done (fused into the next block's dgrad).
        ``fuse_prev = (bn name, y, (c, mean, rstd))``: the BatchNorm that produced this block's
        input; its reductions are fused into this block's last dgrad (whose result is then
        that BN's output gradient)."""
        if dout_is_de:
            dres = dout
            dc3 = self._bn_apply_bwd(pre + "conv3", dout, c3, m3, r3)
        else:
            dc3, dres = self._bn_bwd(pre + "conv3", dout, out, c3, m3, r3, relu=True, want_dres=True)
        if ds is not None:
            cs_, ms, rs = ds
            dcs, _ = self._bn_bwd(pre + "downsample", dres, None, cs_, ms, rs, relu=False)
            dshort = self._wgrad_dgrad(pre + "downsample", dcs, x_in)
        else:
            dshort = dres
        de2 = self._wgrad_dgrad(pre + "conv3", dc3, a2, bn=self._bn_fused(pre + "conv2", a2, c2, m2, r2))
        dc2 = self._bn_apply_bwd(pre + "conv2", de2, c2, m2, r2)
        de1 = self._wgrad_dgrad(pre + "conv2", dc2, a1, bn=self._bn_fused(pre + "conv1", a1, c1, m1, r1))
        dc1 = self._bn_apply_bwd(pre + "conv1", de1, c1, m1, r1)
        bn = None
        if fuse_prev is not None:
            name, y, (c, m, r) = fuse_prev
            bn = self._bn_fused(name, y, c, m, r)
        return self._wgrad_dgrad(pre + "conv1", dc1, x_in, residual=dshort, bn=bn)

    def sgd_step(self, lr, momentum=0.9, wd=5e-5, gscale=1.0):
        p = self.params
        CN.sgd_momentum_mixed(p.master, p.grad, p.mom, p.bf, lr, momentum, wd, gscale)


def synthetic_imagenet(batch, device, size=224, seed=0, num_classes=NUM_CLASSES):
    g = torch.Generator().manual_seed(seed)
    x = torch.zeros(batch, size, size, IN_CH)
    x[..., :3] = torch.randn(batch, size, size, 3, generator=g)
    y = torch.randint(0, num_classes, (batch,), generator=g, dtype=torch.int32)
    return x.to(BF16).to(device), y.to(device)


# ---------------------------------------------------------------------------
# Checkpoint naming: TF conv kernels HWIO [KH, KW, Cin, Cout] (real input
# channels only), BatchNorm gamma/beta/moving_mean/moving_variance, dense
# kernel [in, out].
# ---------------------------------------------------------------------------
def tf_variables(model: ResNet50, prefix="resnet50/"):
    P = model.params
    out = {}
    for name, cin, cout, k, s, p in P.convs:
        w = P.P(name + ".weight").detach().float().cpu()[:, :k * k * cin].reshape(cout, k, k, cin)
        if name == "conv1":
            w = w[..., :3]  # the image has 3 channels; 5 zero pad channels are not a parameter
        out[prefix + name + "/kernel"] = w.permute(1, 2, 3, 0).contiguous()
        bn = prefix + name + "/bn/"
        out[bn + "gamma"] = P.P(name + ".bn.gamma").detach().cpu()
        out[bn + "beta"] = P.P(name + ".bn.beta").detach().cpu()
        rm, rv = P.running[name]
        out[bn + "moving_mean"] = rm.detach().cpu()
        out[bn + "moving_variance"] = rv.detach().cpu()
    out[prefix + "fc/kernel"] = P.P("fc.weight").detach().cpu()[:P.num_classes].t().contiguous()
    out[prefix + "fc/bias"] = P.P("fc.bias").detach().cpu()[:P.num_classes]
    return out


def load_tf_variables(model: ResNet50, values, prefix="resnet50/"):
    P = model.params
    for name, cin, cout, k, s, p in P.convs:
        w = torch.as_tensor(values[prefix + name + "/kernel"]).float().permute(3, 0, 1, 2)
        if name == "conv1":
            w = torch.cat([w, w.new_zeros(cout, k, k, cin - w.shape[-1])], -1)
        dst = P.P(name + ".weight")
        dst.zero_()
        dst[:, :k * k * cin] = w.reshape(cout, -1).to(dst.device)
        bn = prefix + name + "/bn/"
        P.P(name + ".bn.gamma").copy_(torch.as_tensor(values[bn + "gamma"]))
        P.P(name + ".bn.beta").copy_(torch.as_tensor(values[bn + "beta"]))
        rm, rv = P.running[name]
        rm.copy_(torch.as_tensor(values[bn + "moving_mean"]))
        rv.copy_(torch.as_tensor(values[bn + "moving_variance"]))
    fw = P.P("fc.weight")
    fw.zero_()
    fw[:P.num_classes] = torch.as_tensor(values[prefix + "fc/kernel"]).t().to(fw.device)
    fb = P.P("fc.bias")
    fb.zero_()
    fb[:P.num_classes] = torch.as_tensor(values[prefix + "fc/bias"]).to(fb.device)
    TR.cast_bf16(P.master, P.bf)
