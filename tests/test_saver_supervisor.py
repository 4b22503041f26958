"""Saver/FastSaver (utils.py:28-32), checkpoint state, Supervisor (worker.py:107-123)."""
import os
import threading
import time

import numpy as np
import pytest
import torch

from distributedtensorflowexample_amd.train.saver import (FastSaver, Saver, get_checkpoint_state,
                                                          latest_checkpoint, list_variables,
                                                          load_checkpoint)
from distributedtensorflowexample_amd.train.supervisor import Supervisor
from distributedtensorflowexample_amd.utils.summary import FileWriter, merge, read_events, scalar


def _vars():
    return {"global/dense/kernel": torch.randn(784, 100), "global/dense/bias": torch.zeros(100),
            "global/dense_1/kernel": torch.randn(100, 10), "global/dense_1/bias": torch.zeros(10),
            "global/global_step": torch.tensor(42, dtype=torch.int32)}


def test_saver_roundtrip_state_file_and_gc(tmp_path):
    v = _vars()
    s = Saver(v, max_to_keep=5)
    for step in range(1, 8):
        p = s.save(None, str(tmp_path / "model.ckpt"), global_step=step)
    assert p.endswith("model.ckpt-7")
    st = get_checkpoint_state(str(tmp_path))
    assert st.model_checkpoint_path == str(tmp_path / "model.ckpt-7")
    assert [os.path.basename(x) for x in st.all_model_checkpoint_paths] == \
        ["model.ckpt-%d" % i for i in range(3, 8)]
    text = open(tmp_path / "checkpoint").read()
    assert 'model_checkpoint_path: "model.ckpt-7"' in text          # relative, like TF
    assert not os.path.exists(tmp_path / "model.ckpt-2.index")     # max_to_keep = 5
    assert os.path.exists(tmp_path / "model.ckpt-7.meta.json")     # Saver writes a meta
    assert latest_checkpoint(str(tmp_path)) == str(tmp_path / "model.ckpt-7")
    r = load_checkpoint(latest_checkpoint(str(tmp_path)))
    for k, t in v.items():
        assert torch.equal(r[k], t) and r[k].dtype == t.dtype
    assert list_variables(p)[0] == ("global/dense/bias", [100])


def test_fastsaver_never_writes_meta_and_restore_assigns(tmp_path):
    got = {}
    s = FastSaver(_vars(), assign=got.update)
    p = s.save(None, str(tmp_path / "model.ckpt"), global_step=torch.tensor(5))
    assert not os.path.exists(p + ".meta.json")
    s.restore(None, p)
    assert set(got) == set(_vars())
    with pytest.raises(KeyError):
        Saver({"missing": torch.zeros(1)}).restore(None, p)


def test_saver_dtypes(tmp_path):
    v = {"a": torch.randn(3).to(torch.bfloat16), "b": torch.arange(4, dtype=torch.int64),
         "c": torch.randn(2, 2, dtype=torch.float64), "d": np.ones(3, np.float32)}
    p = Saver(v).save(None, str(tmp_path / "x"))
    r = load_checkpoint(p)
    assert r["a"].dtype == torch.bfloat16 and torch.equal(r["a"], v["a"])
    assert torch.equal(r["b"], v["b"]) and torch.equal(r["c"], v["c"])


def test_supervisor_chief_init_then_restore(tmp_path):
    state = {"w": None, "step": 0, "inits": 0}

    def init():
        state["w"], state["inits"] = torch.ones(3), state["inits"] + 1

    def assign(vals):
        state["w"], state["step"] = vals["w"].clone(), int(vals["step"])

    def vars_():
        return {"w": state["w"], "step": torch.tensor(state["step"], dtype=torch.int32)}

    saver = FastSaver({"w": None, "step": None}, assign=assign)
    sv = Supervisor(is_chief=True, logdir=str(tmp_path), saver=saver, init_op=init,
                    global_step=lambda: state["step"], save_model_secs=0.05,
                    save_variables=vars_)
    with sv.managed_session():
        for i in range(5):
            state["step"] += 1
            state["w"] = state["w"] * 2
            time.sleep(0.04)
    assert state["inits"] == 1 and latest_checkpoint(str(tmp_path)) is not None
    saved_step = int(load_checkpoint(latest_checkpoint(str(tmp_path)))["step"])
    assert saved_step >= 1
    state.update(w=None, step=0)
    sv2 = Supervisor(is_chief=True, logdir=str(tmp_path), saver=saver, init_op=init,
                     global_step=lambda: state["step"], save_model_secs=0)
    with sv2.managed_session():
        pass
    assert state["inits"] == 1 and state["step"] == saved_step   # restored, not re-init
    assert sv2.restored_from == latest_checkpoint(str(tmp_path))


def test_supervisor_non_chief_waits_for_ready():
    ready = {"uninit": ["global/w"]}
    sv = Supervisor(is_chief=False, ready_op=lambda: list(ready["uninit"]),
                    recovery_wait_secs=0.02, ready_timeout_secs=5)
    t = threading.Timer(0.1, lambda: ready.update(uninit=[]))
    t.start()
    t0 = time.time()
    with sv.managed_session():
        waited = time.time() - t0
    assert waited >= 0.09
    sv3 = Supervisor(is_chief=False, ready_op=lambda: ["x"], recovery_wait_secs=0.01,
                     ready_timeout_secs=0.05)
    with pytest.raises(TimeoutError):
        with sv3.managed_session():
            pass


def test_supervisor_step_rate_summary(tmp_path):
    w = FileWriter(str(tmp_path), flush_secs=0.05)
    st = {"s": 0}
    sv = Supervisor(is_chief=True, summary_writer=w, global_step=lambda: st["s"],
                    save_summaries_secs=0.05)
    with sv.managed_session():
        for _ in range(10):
            st["s"] += 10
            time.sleep(0.02)
    ev = read_events(w.path)
    rates = [e["scalars"]["global_step/sec"] for e in ev if "global_step/sec" in e["scalars"]]
    assert rates and max(rates) > 0


def test_summary_merge_and_writer(tmp_path):
    s = merge([scalar("loss", 1.0), scalar("accuracy", 0.5)])
    with FileWriter(str(tmp_path)) as w:
        w.add_summary(s, 3)
        w.add_summary({"loss": 0.25}, 4)
    ev = read_events(w.path)
    assert ev[1]["scalars"] == {"loss": 1.0, "accuracy": 0.5} and ev[2]["step"] == 4
