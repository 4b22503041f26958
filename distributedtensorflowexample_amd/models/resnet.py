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
  costs one finalize + one fused apply(+residual +ReLU) pass -- or none of its
  own where the consumer forms it: a bottleneck's output relu(bn3(c3) + shortcut)
  inside the next block's narrow 1x1 conv1 (``_finish_block``), BN3's backward
  apply inside conv3's narrow data gradient (``_block_bwd``), and the stem's
  relu(bn(c)) inside the max pool, forward and backward (never stored);
* flat f32 master / bf16 working copy / f32 gradient / momentum buffers with
  64-element aligned slots; one all-reduce bucket per bottleneck block,
  released as soon as that block's backward finishes;
* the 3-channel input is stored with 8 channels (zero padded) so every
  gather moves 16-byte vectors; the 1000-way classifier is padded to 1024
  output rows (zero weights, masked in the loss).
"""
from __future__ import annotations

import math
import os

import torch

from ..ops import bf16 as B16
from ..ops import cnn as CN
from ..ops import init as I
from ..ops import transformer as TR

BF16 = torch.bfloat16
ALIGN = 64
# the stem's BatchNorm + ReLU fused into its max pool (DTFX_STEM_POOL_BN=0: separate passes)
_STEM_POOL_BN = os.environ.get("DTFX_STEM_POOL_BN", "1") != "0"
_DS_PRO = os.environ.get("DTFX_DS_PROLOGUE", "1") != "0"  # stride-1 downsample BN apply in its dgrad
_DS_COMPACT = os.environ.get("DTFX_DS_COMPACT", "1") != "0"  # stride-2 downsample dgrad kept compact
# the 1x1 data gradients' transposed weights from one batched launch per step
# (DTFX_RESNET_WT_BATCH=0: each dgrad transposes its own)
_WT_BATCH = os.environ.get("DTFX_RESNET_WT_BATCH", "1") != "0"
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
    def __init__(self, device, seed=0, stages=STAGES, num_classes=NUM_CLASSES,
                 bucket_multiple=ALIGN):
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
        # a bucket (stem, each bottleneck block, the head) starts and ends on a multiple of
        # ``bucket_multiple`` elements: the owner-sharded optimizer splits every bucket into W
        # equal, ALIGN-aligned shards (trainer zero1: bucket_multiple = ALIGN * world)
        bm = int(bucket_multiple)
        if bm % ALIGN:
            raise ValueError("bucket_multiple must be a multiple of %d" % ALIGN)

        def opens_bucket(name):
            return name == "fc.weight" or (name.endswith(".conv1.weight") and name != "conv1.weight")

        for name, shape, _ in layout:
            if opens_bucket(name):
                off = (off + bm - 1) // bm * bm
            self.offsets[name] = (off, shape)
            off += (math.prod(shape) + ALIGN - 1) // ALIGN * ALIGN
        off = (off + bm - 1) // bm * bm
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

    def __init__(self, device, seed=0, stages=STAGES, num_classes=NUM_CLASSES, bn_eps=1e-5,
                 bucket_multiple=ALIGN):
        self.device = torch.device(device)
        self.params = ResNetParams(device, seed, stages, num_classes, bucket_multiple)
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
        self._wt = {}        # 1x1 conv name -> its persistent transposed bf16 weight copy
        self._wt_tab = None  # (int64 table, n, tiles) of the per-step batched transpose
        self._fold = False   # enable_splitk_fold
        self._planes = {}    # conv name -> its persistent split-K planes (0: not folded)
        self._segs = None    # the optimizer's segment table (int64 [n][5])

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

    def forward_backward(self, images, labels, on_bucket_ready=None, on_bucket_needed=None):
        """images: NHWC bf16 [N, H, W, 8]; labels int32 [N].  Returns (loss, accuracy).
        ``on_bucket_needed(b)``: called before the forward first reads bucket b's parameters
        (the owner-sharded optimizer waits there for that bucket's all-gather)."""
        P = self.params
        N = images.shape[0]
        need = on_bucket_needed if on_bucket_needed is not None else (lambda b: None)
        P.grad.zero_()
        self._stats_flat.zero_()  # every BN's (sum, sum of squares) accumulators, one memset
        saved = {}
        need(0)
        c, st = self._conv_bn("conv1", images)
        if c.is_cuda and _STEM_POOL_BN:
            # the stem's relu(bn(c)) is formed inside the pool and never stored
            rm, rv = P.running["conv1"]
            x, idx, m, r, fco = CN.bn_maxpool_fwd(c, st[0], st[1], st[2], P.P("conv1.bn.gamma"),
                                                  P.P("conv1.bn.beta"), self.eps, rm, rv)
            saved["conv1"] = (images, c, m, r, None, fco)
        else:
            a, m, r = self._bn_apply("conv1", c, st)
            saved["conv1"] = (images, c, m, r, a, None)
            x, idx = CN.maxpool_fwd(a)
        blocks = []
        pend = None  # the previous block, its output not formed yet (see _finish_block)
        for si, (w, nb, st_) in enumerate(P.stages):
            for b in range(nb):
                pre = "layer%d.%d." % (si + 1, b)
                need(len(blocks) + 1)  # this block's bucket (its conv1 runs next)
                if pend is None:
                    x_in = x
                    c1, s1 = self._conv_bn(pre + "conv1", x_in)
                else:
                    x_in, c1, s1 = self._finish_block(blocks, pend, pre + "conv1")
                n2 = pre + "conv2"
                if CN.bn_relu_conv3x3_applies(c1, P.W(n2 + ".weight")) and self.specs[n2][4] == 1:
                    # layer1: relu(bn1(c1)) formed in the 64-channel 3x3 kernel's patch staging
                    cs, cq, M1 = s1
                    ncs, ncq = self._stats[n2]
                    rm, rv = P.running[pre + "conv1"]
                    a1, c2, m1, r1 = CN.bn_relu_conv3x3(
                        c1, cs, cq, M1, P.P(pre + "conv1.bn.gamma"), P.P(pre + "conv1.bn.beta"),
                        P.W(n2 + ".weight"), ncs, ncq, self.eps, rm, rv)
                    s2 = (ncs, ncq, c2.numel() // c2.shape[-1])
                else:
                    a1, m1, r1 = self._bn_apply(pre + "conv1", c1, s1)
                    c2, s2 = self._conv_bn(n2, a1)
                a2, m2, r2, c3, s3 = self._bn_relu_conv(pre + "conv2", c2, s2, pre + "conv3")
                # (first block: the downsample conv of the same input; its BatchNorm is applied
                # with bn3's, the normalised shortcut is never materialised)
                dsc = self._conv_bn(pre + "downsample", x_in) if b == 0 else None
                blocks.append([pre, x_in, (c1, m1, r1, a1), (c2, m2, r2, a2), None, None, None])
                pend = (len(blocks) - 1, c3, s3, dsc)
        x, _, _ = self._finish_block(blocks, pend, None)
        pooled = CN.avgpool_fwd(x)                               # [N, 2048]
        need(len(P.buckets) - 1)
        logits = B16.gemm(pooled, P.W("fc.weight"), False, True, bias=P.P("fc.bias"),
                          out_dtype=torch.float32)                # [N, 1024]
        loss_rows, correct, dlog = TR.mlm_xent(logits, labels, P.num_classes, 1.0 / N)
        loss = loss_rows.sum() / N
        acc = correct.sum() / N
        # ---------------- backward
        self._transpose_weights()  # the 1x1 data gradients' transposed weights, one launch
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
        img, c, m, r, a, fco = saved["conv1"]
        _, cin, cout, k, s, p = self.specs["conv1"]
        if a is None and CN.stem_wgrad_bn_applies(img, cout, k, s, p):
            # the stem weight gradient forms dL/dc from de and c as it stages them
            de, bco = CN.maxpool_bn_bwd(dx, idx, c, m, r, P.P("conv1.bn.gamma"),
                                        P.P("conv1.bn.beta"), fco, P.G("conv1.bn.gamma"),
                                        P.G("conv1.bn.beta"), apply=False)
            CN.conv_wgrad(de, img, P.G("conv1.weight"), k, k, s, p, beta=1.0, bn_in=(c, bco))
            dc = de
        elif a is None:
            dc = CN.maxpool_bn_bwd(dx, idx, c, m, r, P.P("conv1.bn.gamma"), P.P("conv1.bn.beta"),
                                   fco, P.G("conv1.bn.gamma"), P.G("conv1.bn.beta"))
            CN.conv_wgrad(dc, img, P.G("conv1.weight"), k, k, s, p, beta=1.0)
        else:
            da = CN.maxpool_bwd(dx, idx, a.shape)
            dc, _ = CN.bn_bwd(da, a, c, m, r, P.P("conv1.bn.gamma"), P.G("conv1.bn.gamma"),
                              P.G("conv1.bn.beta"), relu=True, grads_zeroed=True)
            CN.conv_wgrad(dc, img, P.G("conv1.weight"), k, k, s, p, beta=1.0)
        if ws is not None:  # join: every gradient final on the main stream
            torch.cuda.current_stream(dc.device).wait_stream(ws)
            self._keep.clear()
        if on_bucket_ready is not None:
            on_bucket_ready(0)
        return loss, acc

    def _bn_relu_conv(self, name, c, st, next_conv):
        """``a = relu(bn(c))`` and the 1x1 expansion ``next_conv`` of it: one pass over c on the
        wide 1x1 kernel's prologue (``CN.bn_relu_conv1x1``) when it takes the product, else
        bn_apply then the conv.  Returns (a, mean, rstd, y, y statistics)."""
        P = self.params
        cout = self.specs[next_conv][2]
        if CN.bn_prologue_applies(c, c.shape[-1], cout, 3):
            cs, cq, M = st
            ncs, ncq = self._stats[next_conv]
            rm, rv = P.running[name]
            a, y, m, r = CN.bn_relu_conv1x1(c, cs, cq, M, P.P(name + ".bn.gamma"),
                                            P.P(name + ".bn.beta"), P.W(next_conv + ".weight"),
                                            ncs, ncq, self.eps, rm, rv)
            return a, m, r, y, (ncs, ncq, y.numel() // cout)
        a, m, r = self._bn_apply(name, c, st)
        y, sy = self._conv_bn(next_conv, a)
        return a, m, r, y, sy

    def _finish_block(self, blocks, pend, next_conv):
        """Form block ``pend``'s output ``out = relu(bn3(c3) + shortcut)`` (shortcut: the
        block input, or bn_ds(downsample conv output) for a first block) and, with
        ``next_conv`` (the next block's conv1, 1x1 / stride 1), that conv's output.  When the
        narrow 1x1 kernel takes the product, ``out`` is formed inside its prologue
        (``CN.bn_out_conv1x1``: one pass over c3 and the shortcut instead of a bn_apply pass and
        the conv's read of its result); otherwise bn_apply then the conv.  Fills the block's
        (c3, mean, rstd), downsample and output entries.  Returns (out, c1, c1 statistics)."""
        i, c3, s3, dsc = pend
        P = self.params
        pre = blocks[i][0]
        name = pre + "conv3"
        res_bn = None
        residual = blocks[i][1]
        if dsc is not None:
            residual, sds = dsc
            rm, rv = P.running[pre + "downsample"]
            nd = pre + "downsample.bn."
            res_bn = (sds[0], sds[1], P.P(nd + "gamma"), P.P(nd + "beta"), rm, rv)
        c1 = s1 = None
        if next_conv is not None and CN.bn_prologue_applies(c3, c3.shape[-1],
                                                            self.specs[next_conv][2], 1):
            cout = self.specs[next_conv][2]
            cs, cq, M = s3
            ncs, ncq = self._stats[next_conv]
            rm3, rv3 = P.running[name]
            r = CN.bn_out_conv1x1(c3, cs, cq, M, P.P(name + ".bn.gamma"), P.P(name + ".bn.beta"),
                                  residual, P.W(next_conv + ".weight"), ncs, ncq, self.eps, rm3,
                                  rv3, res_bn=res_bn)
            out, c1, stats = r[0], r[1], r[2:]
            s1 = (ncs, ncq, c1.numel() // cout)
        else:
            r = self._bn_apply(name, c3, s3, residual=residual, relu=True, res_bn=res_bn)
            out, stats = r[0], r[1:]
            if next_conv is not None:
                c1, s1 = self._conv_bn(next_conv, out)
        blocks[i][4] = (c3, stats[0], stats[1])
        blocks[i][5] = (residual, stats[2], stats[3]) if dsc is not None else None
        blocks[i][6] = out
        return out, c1, s1

    def _bn_bwd(self, name, dy, y, x, mean, rstd, relu=True, want_dres=False, apply=True):
        P = self.params
        return CN.bn_bwd(dy, y, x, mean, rstd, P.P(name + ".bn.gamma"), P.G(name + ".bn.gamma"),
                         P.G(name + ".bn.beta"), relu, want_dres, grads_zeroed=True, apply=apply)

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

    def _conv1_pro_wide(self, pre, c1, x_in):
        """conv1's data gradient runs on the wide 1x1 kernel with the BN prologue (the path
        that can read a compact stride-2 residual)."""
        K, N = c1.shape[-1], x_in.shape[-1]
        return (CN.bn_prologue_applies(c1, K, N, 2)
                and not CN.hip().conv1x1_pro_applies(1, c1.numel() // K, K, N))

    def enable_splitk_fold(self):
        """Leave the split-K weight gradients as their partial planes and let momentum SGD sum
        them (one GPU only: with data parallelism the bucket all-reduce needs the reduced
        gradient).  Removes the reduce pass of every split weight-gradient launch (49 per
        ResNet-50 step) -- it wrote the f32 gradient only for SGD to read it back.  The planes
        are allocated at each conv's first backward (its shape is known then: the first,
        eager step) and kept; ``p.grad`` no longer holds these gradients
        (:meth:`materialize_grads` sums them there on demand)."""
        if self.device.type != "cuda":
            return False
        self._fold = True
        return True

    def _fold_planes(self, name, x_in, cout, k, s, p):
        if not self._fold:
            return None
        if name not in self._planes:
            P = self.params
            off, (rows, ldw) = P.offsets[name + ".weight"]
            n = CN.wgrad_fold_planes(tuple(x_in.shape), cout, k, k, s, p, ldw)
            self._planes[name] = None
            if n > 0 and len([v for v in self._planes.values() if v is not None]) < 128:
                S = n // (rows * ldw)
                buf = torch.zeros(n, device=self.device)
                self._planes[name] = (buf, off, rows * ldw, S)
                rows_ = sorted((o // 4, (o + m) // 4, b.data_ptr(), m // 4, S_)
                               for b, o, m, S_ in (v for v in self._planes.values() if v))
                self._segs = torch.tensor(rows_, dtype=torch.int64, device=self.device)
        v = self._planes[name]
        return None if v is None else v[0]

    def _wt_for(self, name):
        """The 1x1 conv's transposed weights for its data gradient, formed by the one batched
        transpose at the start of the backward (``None`` the first time a conv asks: it is
        registered then and its own launch transposes this once)."""
        if self.device.type != "cuda" or not _WT_BATCH:
            return None
        if name in self._wt:
            return self._wt[name]
        P = self.params
        w = P.W(name + ".weight")
        cout, cin = self.specs[name][2], self.specs[name][1]
        buf = torch.empty(cin, cout, device=self.device, dtype=w.dtype)
        self._wt[name] = buf
        rows, tiles = [], 0
        for n_, b in self._wt.items():
            src = P.W(n_ + ".weight")
            r, c = self.specs[n_][2], self.specs[n_][1]
            rows.append((src.data_ptr(), b.data_ptr(), r, c, src.stride(0), tiles))
            tiles += ((r + 31) // 32) * ((c + 31) // 32)
        self._wt_tab = (torch.tensor(rows, dtype=torch.int64, device=self.device), len(rows),
                        tiles)
        return None

    def _transpose_weights(self):
        """Start of the backward: every registered 1x1 weight transposed in ONE launch (the bf16
        working copy is final for this step)."""
        if self._wt_tab is not None:  # (the convs registered so far; a new one transposes itself)
            tab, n, tiles = self._wt_tab
            CN.hip().transpose_bf16_batch(tab.data_ptr(), n, tiles, CN.stream_handle())

    def materialize_grads(self):
        """Sum the folded split-K planes into ``params.grad`` (tests, debugging)."""
        P = self.params
        for name, v in self._planes.items():
            if v is None:
                continue
            buf, off, m, S = v
            P.grad[off:off + m] = buf.view(S, m).sum(0)
        return P.grad

    def _wgrad_dgrad(self, name, dc, x_in, residual=None, need_dx=True, bn=None):
        P = self.params
        _, cin, cout, k, s, p = self.specs[name]
        ws = self.wgrad_stream
        planes = self._fold_planes(name, x_in, cout, k, s, p)
        if ws is None:
            CN.conv_wgrad(dc, x_in, P.G(name + ".weight"), k, k, s, p, beta=1.0, planes=planes)
        else:  # weight gradient beside the data gradient (operands kept alive until the join)
            ws.wait_stream(torch.cuda.current_stream(dc.device))
            with torch.cuda.stream(ws):
                CN.conv_wgrad(dc, x_in, P.G(name + ".weight"), k, k, s, p, beta=1.0,
                              planes=planes)
            self._keep.append((dc, x_in))
        if not need_dx:
            return None
        wt = self._wt_for(name) if k == 1 and s == 1 and p == 0 else None
        return CN.conv_dgrad(dc, P.W(name + ".weight"), x_in.shape, k, k, s, p, residual=residual,
                             bn=bn, wt=wt)

    def _block_bwd(self, pre, dout, x_in, c1, m1, r1, a1, c2, m2, r2, a2, c3, m3, r3, ds, out,
                   dout_is_de=False, fuse_prev=None):
        """Backward of one bottleneck.  ``dout_is_de``: ``dout`` is already the gradient at
        conv3's BN output with its reductions done (fused into the next block's dgrad).
        ``fuse_prev = (bn name, y, (c, mean, rstd))``: the BatchNorm that produced this block's
        input; its reductions are fused into this block's last dgrad (whose result is then
        that BN's output gradient)."""
        P = self.params
        n3 = pre + "conv3"
        # conv3's data gradient (a narrow 1x1 product) forms dc3 = BN3-backward(de3) in its
        # prologue when it can: one pass over de3 and c3 (dc3 written for the weight gradient)
        pro = dout_is_de and CN.bn_prologue_applies(c3, c3.shape[-1], a2.shape[-1], 2)
        dc3 = None
        short_s2 = False  # dshort stored compact (stride-2 downsample, see below)
        if dout_is_de:
            dres = dout
            if not pro:
                dc3 = self._bn_apply_bwd(n3, dout, c3, m3, r3)
        else:
            dc3, dres = self._bn_bwd(n3, dout, out, c3, m3, r3, relu=True, want_dres=True)
        if ds is not None:
            cs_, ms, rs = ds
            nd = pre + "downsample"
            if _DS_PRO and self.specs[nd][4] == 1 and CN.bn_prologue_applies(cs_, cs_.shape[-1],
                                                                 x_in.shape[-1], 2):
                # stride-1 downsample (layer1.0): its BN's reductions, then the apply inside the
                # narrow data gradient's prologue (dcs written for the weight gradient)
                self._bn_bwd(nd, dres, None, cs_, ms, rs, relu=False, apply=False)
                dshort, dcs = CN.bn_in_conv1x1_dgrad(dres, cs_, ms, rs, P.P(nd + ".bn.gamma"),
                                                     P.G(nd + ".bn.beta"), P.G(nd + ".bn.gamma"),
                                                     P.W(nd + ".weight"), wt=self._wt_for(nd))
                self._wgrad_dgrad(nd, dcs, x_in, need_dx=False)
            elif (_DS_COMPACT and self.specs[nd][4] == 2 and self._conv1_pro_wide(pre, c1, x_in)
                  and x_in.shape[1] % 2 == 0 and x_in.shape[2] % 2 == 0
                  and x_in.shape[2] >= 16 and x_in.numel() // x_in.shape[-1] < (1 << 24)):
                # stride-2 downsample: its data gradient lives at the even rows / columns only,
                # so it stays compact [N, H/2, W/2, Cin] (a stride-1 1x1 product on the
                # subsampled grid) and conv1's wide data gradient reads it as a stride-2
                # residual -- no full-resolution tensor of mostly zeros written and read back
                dcs, _ = self._bn_bwd(nd, dres, None, cs_, ms, rs, relu=False)
                self._wgrad_dgrad(nd, dcs, x_in, need_dx=False)
                # (a plain [pixels, Cout] x [Cout, Cin] GEMM: 118 / 68 us at layer2.0 / 3.0
                # against 167 / 100 on the conv data-gradient path, tools/probes/ds_compact_gemm.py)
                n_, h_, w_, cin = x_in.shape
                dshort = B16.gemm(dcs.view(-1, dcs.shape[-1]), P.W(nd + ".weight")).view(
                    n_, h_ // 2, w_ // 2, cin)
                short_s2 = True
            else:
                dcs, _ = self._bn_bwd(nd, dres, None, cs_, ms, rs, relu=False)
                dshort = self._wgrad_dgrad(nd, dcs, x_in)
        else:
            dshort = dres
        bn2 = self._bn_fused(pre + "conv2", a2, c2, m2, r2)
        if pro:
            de2, dc3 = CN.bn_in_conv1x1_dgrad(dout, c3, m3, r3, P.P(n3 + ".bn.gamma"),
                                              P.G(n3 + ".bn.beta"), P.G(n3 + ".bn.gamma"),
                                              P.W(n3 + ".weight"), bn2, wt=self._wt_for(n3))
            self._wgrad_dgrad(n3, dc3, a2, need_dx=False)
        else:
            de2 = self._wgrad_dgrad(n3, dc3, a2, bn=bn2)
        dc2 = self._bn_apply_bwd(pre + "conv2", de2, c2, m2, r2)
        de1 = self._wgrad_dgrad(pre + "conv2", dc2, a1, bn=self._bn_fused(pre + "conv1", a1, c1, m1, r1))
        n1 = pre + "conv1"
        bn = None
        if fuse_prev is not None:
            name, y, (c, m, r) = fuse_prev
            bn = self._bn_fused(name, y, c, m, r)
        if CN.bn_prologue_applies(c1, c1.shape[-1], x_in.shape[-1], 2):
            # BN1's backward apply inside conv1's data gradient (dc1 written for the wgrad)
            dx, dc1 = CN.bn_in_conv1x1_dgrad(de1, c1, m1, r1, P.P(n1 + ".bn.gamma"),
                                             P.G(n1 + ".bn.beta"), P.G(n1 + ".bn.gamma"),
                                             P.W(n1 + ".weight"), bn, residual=dshort,
                                             residual_s2=short_s2, wt=self._wt_for(n1))
            self._wgrad_dgrad(n1, dc1, x_in, need_dx=False)
            return dx
        assert not short_s2
        dc1 = self._bn_apply_bwd(n1, de1, c1, m1, r1)
        return self._wgrad_dgrad(n1, dc1, x_in, residual=dshort, bn=bn)

    def sgd_step(self, lr, momentum=0.9, wd=5e-5, gscale=1.0):
        p = self.params
        CN.sgd_momentum_mixed(p.master, p.grad, p.mom, p.bf, lr, momentum, wd, gscale,
                              segs=self._segs)


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
