"""Variable registry (get_vars, utils.py:3-8) and models other than the reference MLP on the
async-PS path (CPU)."""
import glob
import re
import socket

import numpy as np
import pytest
import torch

from distributedtensorflowexample_amd import variables as vs
from distributedtensorflowexample_amd.models.dense import DenseClassifier, make_ps_model


def test_registry_collections_scopes_and_layer_names():
    reg = vs.VariableRegistry()
    with reg.as_default():
        with vs.variable_scope("global"):
            DenseClassifier().build_variables()
            vs.create_global_step()
        with vs.variable_scope("local"):
            DenseClassifier().build_variables()
        # worker.py:27-31 keys, in creation order
        assert [v.name for v in vs.get_vars("global", False)] == [
            "global/dense/kernel", "global/dense/bias", "global/dense_1/kernel",
            "global/dense_1/bias", "global/global_step"]
        assert [v.name for v in vs.get_vars("global")] == [
            "global/dense/kernel", "global/dense/bias", "global/dense_1/kernel",
            "global/dense_1/bias"]
        assert [v.shape for v in vs.get_vars("local")] == [(784, 100), (100,), (100, 10), (10,)]
        # tf.get_collection: re.match of the scope (a prefix, or a regex)
        assert len(vs.get_collection(vs.GLOBAL_VARIABLES)) == 9
        assert [v.name for v in vs.get_vars(r".*/dense_1/")] == [
            "global/dense_1/kernel", "global/dense_1/bias", "local/dense_1/kernel",
            "local/dense_1/bias"]
        with pytest.raises(ValueError):
            vs.get_variable("global/dense/kernel", (1,))
    # the default registry is untouched by as_default() blocks
    assert vs.get_vars("global") == [] or all(
        v.name not in ("global/dense/kernel",) for v in vs.get_vars("global"))


def test_reference_mlp_init_matches_init_params():
    """The registry's initializers reproduce models.mlp.init_params (same seed -> same
    weights under the PS worker and the mirrored trainer)."""
    from distributedtensorflowexample_amd.models.mlp import init_params, to_tf_variables

    reg = vs.VariableRegistry()
    with reg.as_default(), vs.variable_scope("global"):
        vars_ = DenseClassifier().build_variables()
    ref = to_tf_variables(init_params("cpu", seed=3))
    for i, v in enumerate(vars_):
        assert torch.equal(v.initial_value(3, i), ref[v.local_name]), v.name


@pytest.mark.parametrize("name,hidden,dims", [("softmax", "", (784, 10)),
                                              ("mlp", "64,32", (784, 64, 32, 10))])
def test_generic_dense_gradients_match_autograd(name, hidden, dims):
    m = make_ps_model(name, hidden, "relu")
    assert m.dims == dims and not m.is_reference_mlp
    reg = vs.VariableRegistry()
    with reg.as_default(), vs.variable_scope("global"):
        vars_ = m.build_variables()
    tf_vals = [v.initial_value(0, i) * (0.05 if v.dtype == "float32" else 1)
               for i, v in enumerate(vars_)]
    local = m.new_local("cpu")
    m.load_local(local, tf_vals)
    x = torch.rand(32, 784)
    y = torch.randint(0, 10, (32,))
    grads, loss, acc = m.grads(local, x, y)
    # plain torch reference in TF layout
    ps = [t.clone().requires_grad_(True) for t in tf_vals]
    h = x
    for i in range(len(ps) // 2):
        h = h @ ps[2 * i] + ps[2 * i + 1]
        if i < len(ps) // 2 - 1:
            h = torch.relu(h)
    ref_loss = torch.nn.functional.cross_entropy(h, y)
    ref = torch.autograd.grad(ref_loss, ps)
    assert abs(loss - float(ref_loss)) < 1e-5
    for g, r, v in zip(grads, ref, vars_):
        assert g.shape == tuple(v.shape)
        assert float((g - r).abs().max()) < 1e-5, v.name


def _free_port_block(n):
    for _ in range(50):
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            base = s.getsockname()[1]
        if base + n < 65000:
            ok = True
            for p in range(base, base + n):
                with socket.socket() as t:
                    try:
                        t.bind(("127.0.0.1", p))
                    except OSError:
                        ok = False
                        break
            if ok:
                return base
    raise RuntimeError("no free port block")


def test_parameter_server_strategy_variable_store_from_get_vars():
    """ParameterServerStrategy.variable_store(get_vars('global', False)) for the reference
    MLP and for softmax regression: the ps holds exactly the registry's variables."""
    from distributedtensorflowexample_amd.cluster import Server
    from distributedtensorflowexample_amd.distribute import ParameterServerStrategy
    from distributedtensorflowexample_amd.train.worker import build_worker_variables

    base = _free_port_block(2)
    spec = {"ps": ["127.0.0.1:%d" % base], "worker": ["127.0.0.1:%d" % (base + 1)]}
    ps = Server(spec, "ps", 0)
    try:
        for k, name in enumerate(("mlp", "softmax")):
            model = make_ps_model(name)
            reg = vs.VariableRegistry()
            with reg.as_default(), vs.variable_scope("job%d" % k):
                with vs.variable_scope("global"):
                    model.build_variables()
                    vs.create_global_step()
                gvars = vs.get_vars("job%d/global" % k, False)
            st = ParameterServerStrategy(spec).variable_store([v.spec for v in gvars]).create()
            st.assign({v.name: (0 if v.dtype != "float32" else v.initial_value(0, i))
                       for i, v in enumerate(gvars)})
            assert st.uninitialized() == []
            got = st.read_all()
            assert sorted(got) == sorted(v.name for v in gvars)
            for i, v in enumerate(gvars):
                if v.dtype == "float32":
                    assert torch.equal(got[v.name], v.initial_value(0, i))
            st.close()
        g, t = build_worker_variables(make_ps_model("softmax"), vs.VariableRegistry())
        assert [v.name for v in g] == ["global/dense/kernel", "global/dense/bias",
                                      "global/global_step"]
        assert [v.name for v in t] == ["global/dense/kernel", "global/dense/bias"]
    finally:
        ps.stop()


@pytest.mark.slow
def test_async_ps_cluster_trains_softmax_regression(tmp_path):
    """main.py --model softmax: 1 ps + 2 CPU workers train a model other than the reference's
    through the same Worker; its checkpoint holds the registry's variables."""
    from distributedtensorflowexample_amd.launch import launch_ps
    from distributedtensorflowexample_amd.train.saver import latest_checkpoint, load_checkpoint

    logdir = str(tmp_path / "sm")
    base = _free_port_block(4)
    rc = launch_ps(num_workers=2, num_gpus=1, num_ps=1, cpu=True, base_port=base,
                   log_dir=str(tmp_path / "logs"), quiet=True, timeout=240,
                   extra=["--model", "softmax", "--training_steps", "600", "--log_every", "100",
                          "--eval_every", "300", "--logdir", logdir, "--save_model_secs", "0.3",
                          "--learning_rate", "0.5"])
    assert rc == {"worker0": 0, "worker1": 0}, rc
    logs = "".join(open(p).read() for p in glob.glob(str(tmp_path / "logs" / "worker*.log")))
    costs = [float(c) for c in re.findall(r"cost: ([0-9.eE+-]+)", logs)]
    accs = [float(a) for a in re.findall(r"test accuracy: ([0-9.]+)", logs)]
    assert costs and accs, logs
    assert max(accs) > 0.6, accs  # softmax regression learns the synthetic digits
    v = load_checkpoint(latest_checkpoint(logdir))
    assert sorted(v) == ["global/dense/bias", "global/dense/kernel", "global/global_step"]
    assert tuple(v["global/dense/kernel"].shape) == (784, 10)
    assert np.isfinite(v["global/dense/kernel"].numpy()).all()
