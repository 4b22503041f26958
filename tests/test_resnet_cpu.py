"""Tiny ResNet (same code path as ResNet-50) on the CPU references vs torch autograd."""
import torch
import torch.nn.functional as F

from distributedtensorflowexample_amd.models.resnet import ResNet50, conv_specs, synthetic_imagenet

STAGES = [(8, 2, 1), (16, 1, 2)]


def _ref(model, x, y):
    P = model.params
    W = {}
    for name, cin, cout, k, s, p in P.convs:
        w = P.P(name + ".weight")[:, :k * k * cin].reshape(cout, k, k, cin).permute(0, 3, 1, 2)
        W[name] = w.clone().requires_grad_(True)
    G = {n: P.P(n).clone().requires_grad_(True) for n, _, _ in P.layout if ".bn." in n}
    fcw = P.P("fc.weight").clone().requires_grad_(True)
    fcb = P.P("fc.bias").clone().requires_grad_(True)

    def cbr(name, h, relu=True, res=None):
        _, cin, cout, k, s, p = model.specs[name]
        c = F.conv2d(h, W[name], stride=s, padding=p)
        o = F.batch_norm(c, None, None, G[name + ".bn.gamma"], G[name + ".bn.beta"], True, 0.0, 1e-5)
        if res is not None:
            o = o + res
        return F.relu(o) if relu else o

    h = x.float().permute(0, 3, 1, 2)
    h = F.max_pool2d(cbr("conv1", h), 3, 2, 1)
    for si, (w, nb, st) in enumerate(P.stages):
        for b in range(nb):
            pre = "layer%d.%d." % (si + 1, b)
            sc = cbr(pre + "downsample", h, relu=False) if b == 0 else h
            t = cbr(pre + "conv2", cbr(pre + "conv1", h))
            h = cbr(pre + "conv3", t, res=sc)
    pooled = h.mean((2, 3))
    logits = pooled @ fcw.t() + fcb
    loss = F.cross_entropy(logits[:, :P.num_classes], y.long())
    loss.backward()
    return loss, W, G, fcw


def test_tiny_resnet_matches_autograd():
    torch.manual_seed(0)
    m = ResNet50("cpu", seed=1, stages=STAGES, num_classes=10)
    x, y = synthetic_imagenet(4, "cpu", size=32, seed=2, num_classes=10)
    loss, acc = m.forward_backward(x, y)
    ref, W, G, fcw = _ref(m, x, y)
    assert abs(loss.item() - ref.item()) < 0.03 * ref.item()
    P = m.params
    for name in ["conv1", "layer1.0.conv2", "layer2.0.downsample", "layer2.0.conv3"]:
        _, cin, cout, k, s, p = m.specs[name]
        g = P.G(name + ".weight")[:, :k * k * cin].flatten()
        r = W[name].grad.permute(0, 2, 3, 1).reshape(-1)
        cos = torch.dot(g, r) / (g.norm() * r.norm() + 1e-30)
        # activations are rounded to bf16 after every op (the reference runs in f32): the
        # agreement decays with depth through the batch-statistics BatchNorm backward
        assert cos > 0.94, (name, cos.item())
    for name in ["layer1.1.conv3.bn.gamma", "conv1.bn.beta"]:
        g, r = P.G(name), G[name].grad
        cos = torch.dot(g, r) / (g.norm() * r.norm() + 1e-30)
        assert cos > 0.94, (name, cos.item())
    g, r = P.G("fc.weight")[:10].flatten(), fcw.grad[:10].flatten()
    assert torch.dot(g, r) / (g.norm() * r.norm()) > 0.99


def test_resnet50_layout():
    specs = conv_specs()
    assert len(specs) == 53  # 1 stem + 16 blocks x 3 + 4 projections
    n = 0
    for name, cin, cout, k, s, p in specs:
        n += cout * k * k * cin + 2 * cout
    n += 2048 * 1000 + 1000
    assert 25.5e6 < n < 25.7e6  # ResNet-50: 25.56 M parameters (3-channel stem: 25.557 M)
