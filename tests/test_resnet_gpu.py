"""ResNet on the GPU kernels vs the same code on the CPU reference paths."""
import pytest
import torch

from distributedtensorflowexample_amd.models.resnet import ResNet50, synthetic_imagenet

pytestmark = pytest.mark.gpu
STAGES = [(64, 2, 1), (128, 1, 2)]


def test_small_resnet_gpu_matches_cpu(gpu):
    mg = ResNet50(gpu, seed=1, stages=STAGES, num_classes=10)
    mc = ResNet50("cpu", seed=1, stages=STAGES, num_classes=10)
    mc.params.master.copy_(mg.params.master.cpu())
    mc.params.bf.copy_(mg.params.bf.cpu())
    x, y = synthetic_imagenet(8, "cpu", size=32, seed=2, num_classes=10)
    lg, _ = mg.forward_backward(x.to(gpu), y.to(gpu))
    lc, _ = mc.forward_backward(x, y)
    assert abs(lg.item() - lc.item()) < 0.02 * lc.item()
    P, Q = mg.params, mc.params
    for name in ["conv1.weight", "layer1.0.conv2.weight", "layer2.0.downsample.weight",
                 "layer1.1.conv3.bn.gamma", "fc.weight"]:
        g, r = P.G(name).cpu().flatten(), Q.G(name).flatten()
        cos = torch.dot(g, r) / (g.norm() * r.norm() + 1e-30)
        assert cos > 0.97, (name, cos.item())


def test_resnet50_trainer_steps(gpu):
    from distributedtensorflowexample_amd.train.resnet_trainer import ResNetTrainer

    tr = ResNetTrainer(64, gpu, image_size=64)
    tr.run(2)
    l0, _ = tr.stats()
    tr.run(3, use_graph=True)
    l1, _ = tr.stats()
    assert 0 < l1 < 15 and l0 > 0


def test_resnet_fits_fixed_batch(gpu):
    from distributedtensorflowexample_amd.train.resnet_trainer import ResNetTrainer

    tr = ResNetTrainer(64, gpu, lr=0.05, image_size=32, stages=STAGES, num_classes=10)
    tr.run(1)
    l0, _ = tr.stats()
    tr.run(24)
    l1, a1 = tr.stats()
    assert l1 < 0.5 * l0, (l0, l1)   # memorises the fixed synthetic batch


def test_resnet_224_resident_weight_kernels_match_cpu(gpu):
    """At 224 x 224 the stem (stem_conv.hip), layer1's 64-channel 3x3 (conv3x3_c64.hip) and
    layer2's stride-1 128-channel 3x3 (conv3x3_c128.hip) kernels run inside the model: loss and
    the gradients that flow through them match the CPU reference path."""
    stages = [(64, 1, 1), (128, 2, 2)]
    mg = ResNet50(gpu, seed=3, stages=stages, num_classes=10)
    mc = ResNet50("cpu", seed=3, stages=stages, num_classes=10)
    mc.params.master.copy_(mg.params.master.cpu())
    mc.params.bf.copy_(mg.params.bf.cpu())
    x, y = synthetic_imagenet(2, "cpu", size=224, seed=4, num_classes=10)
    lg, _ = mg.forward_backward(x.to(gpu), y.to(gpu))
    lc, _ = mc.forward_backward(x, y)
    assert abs(lg.item() - lc.item()) < 0.02 * lc.item()
    P, Q = mg.params, mc.params
    for name in ["conv1.weight", "layer1.0.conv1.weight", "layer1.0.conv2.weight",
                 "layer2.1.conv2.weight", "layer2.0.conv1.weight", "conv1.bn.gamma"]:
        g, r = P.G(name).cpu().flatten(), Q.G(name).flatten()
        cos = torch.dot(g, r) / (g.norm() * r.norm() + 1e-30)
        assert cos > 0.97, (name, cos.item())


def test_resnet_splitk_fold_matches_reduce(gpu):
    """One GPU: the split-K weight gradients stay as their partial planes and momentum SGD sums
    them (ResNet50.enable_splitk_fold, conv_bf16 defer_reduce, sgd_momentum_mixed segments)
    instead of one reduce launch per weight gradient.  Op level: every folded shape's planes
    sum to the reduce path's gradient and to an f32 reference, the SGD with segments equals
    the plain SGD on the reduced gradient; model level: the folded gradients point the same way
    as the reduce path's.  (The model's backward itself is not bit-reproducible run to run --
    BatchNorm reductions use atomics, tools/probes/resnet_grad_determinism.py: up to ~7 % of a
    tensor's max element on its largest outliers -- so the model check is directional.)"""
    from distributedtensorflowexample_amd.ops import cnn as CN

    stages = [(64, 1, 1), (128, 1, 2)]
    x, y = synthetic_imagenet(32, gpu, size=112, seed=5, num_classes=10)
    mf = ResNet50(gpu, seed=6, stages=stages, num_classes=10)
    mr = ResNet50(gpu, seed=6, stages=stages, num_classes=10)
    assert mf.enable_splitk_fold()
    mf.forward_backward(x, y)
    mr.forward_backward(x, y)
    folded = [n for n, v in mf._planes.items() if v is not None]
    assert folded and mf._segs is not None and mf._segs.shape[0] == len(folded)
    gf = mf.materialize_grads().clone()
    for n in folded:
        off, shape = mf.params.offsets[n + ".weight"]
        a, b = gf[off:off + shape[0] * shape[1]], mr.params.grad[off:off + shape[0] * shape[1]]
        assert torch.dot(a, b) / (a.norm() * b.norm()) > 0.99, n
    # op level, deterministic inputs: planes vs the reduce pass vs f32, at two folded shapes
    g = torch.Generator(device=gpu).manual_seed(7)
    for (N, H, W, C, Cout, k, s, p) in [(32, 28, 28, 256, 512, 1, 2, 0), (32, 14, 14, 128, 128, 3, 1, 1)]:
        OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        xi = torch.randn(N, H, W, C, device=gpu, generator=g).to(torch.bfloat16)
        dy = torch.randn(N, OH, OW, Cout, device=gpu, generator=g).to(torch.bfloat16)
        ldw = k * k * C
        n = CN.wgrad_fold_planes(tuple(xi.shape), Cout, k, k, s, p, ldw)
        assert n > 0
        dw = torch.zeros(Cout, ldw, device=gpu)
        CN.conv_wgrad(dy, xi, dw, k, k, s, p, beta=1.0)
        planes = torch.zeros(n, device=gpu)
        untouched = torch.zeros(Cout, ldw, device=gpu)
        CN.conv_wgrad(dy, xi, untouched, k, k, s, p, beta=1.0, planes=planes)
        assert torch.equal(untouched, torch.zeros_like(untouched))
        S = n // (Cout * ldw)
        gsum = planes.view(S, Cout, ldw).sum(0)
        ref = torch.nn.grad.conv2d_weight(xi.float().permute(0, 3, 1, 2), (Cout, C, k, k),
                                          dy.float().permute(0, 3, 1, 2), stride=s,
                                          padding=p).permute(0, 2, 3, 1).reshape(Cout, -1)
        sc = ref.abs().max()
        assert (gsum - ref).abs().max() <= 1e-5 * sc and (dw - ref).abs().max() <= 1e-5 * sc
        # SGD over a flat buffer whose middle range is this gradient's planes
        pad = 256
        tot = pad + Cout * ldw + pad
        p0 = torch.randn(tot, device=gpu, generator=g)
        gr = torch.randn(tot, device=gpu, generator=g)
        gr_red = gr.clone()
        gr_red[pad:pad + Cout * ldw] = dw.view(-1)
        segs = torch.tensor([[pad // 4, (pad + Cout * ldw) // 4, planes.data_ptr(),
                              Cout * ldw // 4, S]], dtype=torch.int64, device=gpu)
        outs = []
        for sg, gg in ((segs, gr), (None, gr_red)):
            pp, v = p0.clone(), torch.full_like(p0, 0.1)
            pb = torch.empty(tot, device=gpu, dtype=torch.bfloat16)
            CN.sgd_momentum_mixed(pp, gg, v, pb, 0.05, 0.9, 5e-5, 0.5, segs=sg)
            outs.append((pp, v))
        for a, b in zip(outs[0], outs[1]):
            assert (a - b).abs().max() <= 1e-6 * b.abs().max(), (N, H, W, C, Cout, k, s, p)
