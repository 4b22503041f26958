"""Flags (main.py:26-39), cluster spec (utils.py:10-26), config (main.py:58-64)."""
import json

import pytest

from distributedtensorflowexample_amd import flags as F
from distributedtensorflowexample_amd.cluster import ClusterSpec, Server, cluster_spec
from distributedtensorflowexample_amd.config import ConfigProto, GPUOptions, memory_fraction


@pytest.fixture
def fv():
    v = F.FlagValues()
    F.define_reference_flags(v)
    return v


def test_reference_defaults(fv):
    fv([])
    d = fv.flag_values_dict()
    assert d["job_name"] == "ps" and d["task_index"] == 0 and d["batch_size"] == 100
    assert d["learning_rate"] == 0.001 and d["training_steps"] == 10 ** 7
    assert d["logdir"] == "./tmp/mnist/1" and d["num_workers"] == 2 and d["num_gpus"] == 1


def test_flag_syntaxes(fv):
    rest = fv(["main.py", "--job_name", "worker", "--task_index=3", "--learning_rate", "0.5",
               "--synthetic", "--nouse_locking", "pos", "--training_steps=1e4"])
    assert fv.job_name == "worker" and fv.task_index == 3 and fv.learning_rate == 0.5
    assert fv.synthetic is True and fv.use_locking is False and fv.training_steps == 10000
    assert rest == ["main.py", "pos"]


def test_unknown_flag_raises(fv):
    with pytest.raises(F.FlagError):
        fv(["m", "--bogus", "1"])
    fv.reset()
    assert fv(["m", "--bogus", "1"], known_only=True)[1:] == ["--bogus", "1"]


def test_bad_value(fv):
    with pytest.raises(F.FlagError):
        fv(["m", "--task_index", "x"])


def test_cluster_spec_single_and_multi_gpu_scripts():
    # run_single_gpu.sh: 1 ps + 2 workers on ports 12222-12224
    assert cluster_spec(2, 1) == {"ps": ["127.0.0.1:12222"],
                                  "worker": ["127.0.0.1:12223", "127.0.0.1:12224"]}
    # run_multi_gpu.sh: 1 ps + 16 workers on 12222-12238
    s = cluster_spec(16, 1)
    assert s["worker"][-1] == "127.0.0.1:12238" and len(s["worker"]) == 16
    s = cluster_spec(2, 3, base_port=5000)
    assert s["ps"] == ["127.0.0.1:5000", "127.0.0.1:5001", "127.0.0.1:5002"]
    assert s["worker"][0] == "127.0.0.1:5003"


def test_cluster_spec_api():
    c = ClusterSpec(cluster_spec(2, 1))
    assert c.jobs == ["ps", "worker"] and c.num_tasks("worker") == 2
    assert c.task_address("worker", 1) == "127.0.0.1:12224"
    assert c.job_tasks("ps") == ["127.0.0.1:12222"]
    assert ClusterSpec(c) == c and ClusterSpec(c.as_dict()) == c
    with pytest.raises(ValueError):
        c.task_address("worker", 7)
    env = json.dumps({"cluster": {"ps": ["h:1"], "worker": ["h:2", "h:3"]},
                      "task": {"type": "worker", "index": 1}})
    c2, t, i = ClusterSpec.from_tf_config(env)
    assert c2.num_tasks("worker") == 2 and t == "worker" and i == 1


def test_memory_fraction_matches_reference():
    assert memory_fraction(2, 1) == pytest.approx(0.45)     # run_single_gpu.sh
    assert memory_fraction(16, 4) == pytest.approx(0.225)   # run_multi_gpu.sh
    cfg = ConfigProto(GPUOptions(per_process_gpu_memory_fraction=0.45))
    assert cfg.apply() is cfg


def test_ps_server_starts_on_its_address():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    spec = {"ps": ["127.0.0.1:%d" % port], "worker": ["127.0.0.1:1"]}
    srv = Server(spec, "ps", 0)
    try:
        assert srv.port == port
        w = Server(spec, "worker", 0)
        assert w.target == ["127.0.0.1:%d" % port]
    finally:
        srv.stop()


def test_gpu_parameter_store_flag_validation(fv):
    """--ps_device gpu: parsed like the reference's flags; a worker that cannot run the
    device store (CPU worker, or with --sync_replicas) is refused before touching the ps."""
    import types

    from distributedtensorflowexample_amd.train.worker import Worker

    fv(["main.py", "--ps_device", "gpu"])
    assert fv.ps_device == "gpu"
    spec = {"ps": ["127.0.0.1:1"], "worker": ["127.0.0.1:2"]}
    fl = types.SimpleNamespace(batch_size=100, learning_rate=0.001, ps_device="gpu",
                               num_workers=1, sync_replicas=False, logdir="unused")
    with pytest.raises(ValueError, match="ps_device gpu"):
        Worker("worker", 0, Server(spec, "worker", 0, start=False), fl, device="cpu")
