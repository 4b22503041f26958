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
