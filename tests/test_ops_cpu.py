"""CPU paths of the ops (the CPU tier / plumbing config) vs plain autograd."""
import torch

from distributedtensorflowexample_amd.models.mlp import MnistMLP, from_tf_variables, init_params, \
    to_tf_variables
from distributedtensorflowexample_amd.ops import init, mlp_step, nn, optim


def test_dense_and_xent_cpu_match_autograd():
    torch.manual_seed(0)
    x = torch.randn(20, 30, dtype=torch.float64, requires_grad=True)
    w = torch.randn(7, 30, dtype=torch.float64, requires_grad=True)
    b = torch.randn(7, dtype=torch.float64, requires_grad=True)
    y = torch.randint(0, 7, (20,))
    loss, acc = nn.softmax_cross_entropy(nn.dense(x, w, b, "sigmoid"), y)
    loss.backward()
    ref = [t.detach().clone().requires_grad_() for t in (x, w, b)]
    l2 = torch.nn.functional.cross_entropy(torch.sigmoid(ref[0] @ ref[1].t() + ref[2]), y)
    l2.backward()
    assert abs(loss.item() - l2.item()) < 1e-10
    for t, r in zip((x, w, b), ref):
        assert torch.allclose(t.grad, r.grad, atol=1e-10)


def test_dense_labels_cpu():
    logits = torch.randn(5, 4, dtype=torch.float64)
    lab = torch.nn.functional.one_hot(torch.tensor([0, 1, 2, 3, 0]), 4).double()
    l, d, c = nn.softmax_xent_stats(logits, lab)
    ref = torch.nn.functional.cross_entropy(logits, lab.argmax(1), reduction="none")
    assert torch.allclose(l, ref)


def test_mlp_reference_step_matches_autograd():
    p = init_params("cpu", seed=3).double() * 0.1
    x = torch.rand(16, 784, dtype=torch.float64)
    y = torch.randint(0, 10, (16,))
    g, loss, acc = mlp_step.reference_step(p, x, y)
    m = MnistMLP(flat=p.clone())
    l2, a2 = m.loss(x, y)
    l2.backward()
    assert abs(loss.item() - l2.item()) < 1e-12
    assert torch.allclose(g, m.flat.grad, atol=1e-12)


def test_tf_variable_layout_roundtrip():
    p = init_params("cpu", seed=1)
    v = to_tf_variables(p)
    assert v["dense/kernel"].shape == (784, 100) and v["dense_1/kernel"].shape == (100, 10)
    q = from_tf_variables(torch.zeros_like(p), v)
    assert torch.equal(p, q)
    # reference init: W ~ N(0, 1), biases 0
    assert abs(float(p[:78400].std()) - 1.0) < 0.02 and float(p[78400:78500].abs().sum()) == 0


def test_optimizers_cpu():
    p, g = torch.ones(10), torch.full((10,), 2.0)
    optim.sgd_(p, g, 0.5)
    assert torch.equal(p, torch.zeros(10))
    m, v = torch.zeros(10), torch.zeros(10)
    optim.adam_(p, g, m, v, 0.1, 1)
    assert torch.allclose(p, torch.full((10,), -0.1), atol=1e-6)


def test_init_cpu_distributions():
    t = torch.empty(100000)
    init.fill_(t, "truncated_normal", 0.0, 1.0, seed=2)
    assert t.abs().max() <= 2.0
    init.fill_(t, "uniform", 2.0, 3.0, seed=2)
    assert 2.0 <= t.min() and t.max() < 3.0


def test_gpu_store_layout_round_trip():
    """The GPU parameter store keeps the fused kernels' flat layout (W stored [out, in]); its
    TF-layout boundary (assign / pull / read_all) round-trips every variable exactly."""
    import torch

    from distributedtensorflowexample_amd.ops import mlp_step
    from distributedtensorflowexample_amd.parallel.gpu_ps import _flat_from_tf, _tf_from_flat

    g = torch.Generator().manual_seed(3)
    tf = {"global/dense/kernel": torch.randn(784, 100, generator=g),
          "global/dense/bias": torch.randn(100, generator=g),
          "global/dense_1/kernel": torch.randn(100, 10, generator=g),
          "global/dense_1/bias": torch.randn(10, generator=g)}
    flat = _flat_from_tf(tf, torch.zeros(mlp_step.NPARAM))
    W1t, _, W2t, _ = mlp_step.unflatten(flat)
    assert torch.equal(W1t, tf["global/dense/kernel"].t())
    assert torch.equal(W2t, tf["global/dense_1/kernel"].t())
    back = _tf_from_flat(flat)
    for k, v in tf.items():
        assert torch.equal(back[k], v), k
        assert back[k].is_contiguous()
