"""End-to-end multi-process runs on CPU (the reference's localhost cluster style).

* async PS: 1 ps + 2 workers through main.py and the launcher (BASELINE config 1:
  "1 ps + 1 worker on localhost CPU", plumbing, no GPU);
* sync DP: 2 ranks over gloo through main.py --strategy mirrored.
"""
import glob
import re
import socket

import pytest

from distributedtensorflowexample_amd.launch import launch_mirrored, launch_ps
from distributedtensorflowexample_amd.train.saver import latest_checkpoint, load_checkpoint
from distributedtensorflowexample_amd.utils.summary import read_events

pytestmark = pytest.mark.slow


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


def test_async_ps_cluster_cpu(tmp_path):
    logdir = str(tmp_path / "mnist")
    base = _free_port_block(4)
    rc = launch_ps(num_workers=2, num_gpus=1, num_ps=1, cpu=True, base_port=base,
                   log_dir=str(tmp_path / "logs"), quiet=True, timeout=240,
                   extra=["--training_steps", "400", "--log_every", "100", "--eval_every", "200",
                          "--logdir", logdir, "--save_model_secs", "0.5",
                          "--learning_rate", "0.01"])
    assert rc == {"worker0": 0, "worker1": 0}, rc
    logs = "".join(open(p).read() for p in glob.glob(str(tmp_path / "logs" / "worker*.log")))
    assert "Per-process GPU memory fraction: 0.45" in logs
    costs = [float(c) for c in re.findall(r"cost: ([0-9.eE+-]+)", logs)]
    assert costs, logs
    assert "test accuracy:" in logs
    # chief checkpoints carry the reference's variable names
    ck = latest_checkpoint(logdir)
    assert ck is not None
    v = load_checkpoint(ck)
    assert sorted(v) == ["global/dense/bias", "global/dense/kernel", "global/dense_1/bias",
                         "global/dense_1/kernel", "global/global_step"]
    assert tuple(v["global/dense/kernel"].shape) == (784, 100)
    # the chief wrote the graph (TF Supervisor): graph.pbtxt in logdir + a graph_def event
    assert open(logdir + "/graph.pbtxt").read().count('op: "ApplyGradientDescent"') == 4
    ev0 = read_events(glob.glob(logdir + "_0/events.out.tfevents.*")[0])
    assert sum("graph_def" in e for e in ev0) == 1
    # per-worker TensorBoard files with loss/accuracy every step
    for t in (0, 1):
        ev = read_events(glob.glob(logdir + "_%d/events.out.tfevents.*" % t)[0])
        tags = set().union(*[e["scalars"].keys() for e in ev])
        assert {"loss", "accuracy"} <= tags
    # both workers contributed: global steps are unique across workers
    steps = []
    for t in (0, 1):
        ev = read_events(glob.glob(logdir + "_%d/events.out.tfevents.*" % t)[0])
        steps += [e["step"] for e in ev if "loss" in e["scalars"]]
    assert len(steps) == len(set(steps))


def test_sync_replicas_ps_cluster_cpu(tmp_path):
    """main.py --sync_replicas (tf.train.SyncReplicasOptimizer): 1 ps + 2 workers; every step
    is ONE averaged apply, so global_step counts rounds (not pushes) and both workers log the
    same steps."""
    logdir = str(tmp_path / "sync")
    base = _free_port_block(4)
    rc = launch_ps(num_workers=2, num_gpus=1, num_ps=1, cpu=True, base_port=base,
                   log_dir=str(tmp_path / "logs"), quiet=True, timeout=240,
                   extra=["--training_steps", "200", "--log_every", "50", "--eval_every", "100",
                          "--logdir", logdir, "--save_model_secs", "0.2", "--sync_replicas",
                          "--learning_rate", "0.05"])
    assert rc == {"worker0": 0, "worker1": 0}, rc
    v = load_checkpoint(latest_checkpoint(logdir))  # the chief's periodic saves
    assert 0 < int(v["global/global_step"]) <= 201  # rounds 0..200, one apply each
    steps = []
    for t in (0, 1):
        log = open(str(tmp_path / "logs" / ("worker%d.log" % t))).read()
        steps.append(re.findall(r"step: (\d+)", log))
    assert steps[0] == steps[1] == ["50", "100", "150", "200"], steps


def test_mirrored_two_ranks_gloo(tmp_path):
    logdir = str(tmp_path / "mir")
    rc = launch_mirrored(nproc=2, log_dir=str(tmp_path / "logs"), quiet=True, timeout=240,
                         extra=["--training_steps", "300", "--log_every", "100",
                                "--eval_every", "300", "--logdir", logdir, "--device", "cpu",
                                "--learning_rate", "0.05", "--save_model_secs", "100"])
    assert rc == {"rank0": 0, "rank1": 0}, rc
    log0 = open(str(tmp_path / "logs" / "rank0.log")).read()
    assert "step: 300" in log0 and "test accuracy:" in log0
    v = load_checkpoint(latest_checkpoint(logdir))
    assert int(v["global/global_step"]) == 300


def test_mirrored_two_ranks_frequent_checkpoints_with_replica_check(tmp_path):
    """A checkpoint timer much faster than the steps plus the replica-identity check every
    10 steps: the chief saves between chunks on its training thread, so the replicas never
    diverge (the check would stop the run) and no rank waits on a collective the other
    never joins."""
    logdir = str(tmp_path / "mir")
    rc = launch_mirrored(nproc=2, log_dir=str(tmp_path / "logs"), quiet=True, timeout=240,
                         extra=["--training_steps", "200", "--log_every", "10",
                                "--eval_every", "200", "--logdir", logdir, "--device", "cpu",
                                "--learning_rate", "0.05", "--save_model_secs", "0.01",
                                "--check_replicas_every", "10"])
    assert rc == {"rank0": 0, "rank1": 0}, rc
    v = load_checkpoint(latest_checkpoint(logdir))
    assert int(v["global/global_step"]) == 200


def test_mirrored_zero1_matches_allreduce(tmp_path):
    """main.py --strategy mirrored --zero1 (reduce-scatter, owner SGD on 1/2 of the
    parameters, all-gather) reaches the same parameters as the all-reduce path."""
    import numpy as np

    out = {}
    for tag, extra in (("ar", []), ("z1", ["--zero1"])):
        logdir = str(tmp_path / tag)
        rc = launch_mirrored(nproc=2, log_dir=str(tmp_path / ("logs_" + tag)), quiet=True,
                             timeout=240,
                             extra=["--training_steps", "60", "--log_every", "30",
                                    "--eval_every", "60", "--logdir", logdir, "--device", "cpu",
                                    "--learning_rate", "0.05", "--save_model_secs", "100"] + extra)
        assert rc == {"rank0": 0, "rank1": 0}, (tag, rc)
        out[tag] = load_checkpoint(latest_checkpoint(logdir))
    assert int(out["z1"]["global/global_step"]) == 60
    for k in ("global/dense/kernel", "global/dense/bias", "global/dense_1/kernel",
              "global/dense_1/bias"):
        a, b = np.asarray(out["ar"][k]), np.asarray(out["z1"][k])
        assert np.abs(a - b).max() < 1e-5, k
