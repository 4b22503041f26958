"""Native host runtime: CRC32C, TF-V2 tensor bundle, TFRecord events, TCP PS.

TF is not installed, so format compatibility is pinned by golden bytes
derived from the format definitions (LevelDB table, tensor_bundle.proto,
TFRecord framing) and published CRC32C test vectors.
"""
import os
import struct
import threading

import numpy as np
import pytest


@pytest.fixture(scope="module")
def h():
    from distributedtensorflowexample_amd.ops import host

    return host()


# ---------------------------------------------------------------- CRC32C
def _mask_py(c):
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def test_crc32c_vectors(h):
    assert h.crc32c(b"123456789") == 0xE3069283          # Castagnoli check value
    assert h.crc32c(b"") == 0
    assert h.crc32c(b"\x00" * 32) == 0x8A9136AA          # RFC 3720 B.4
    assert h.crc32c(b"\xff" * 32) == 0x62A8AB43
    assert h.crc32c(bytes(range(32))) == 0x46DD794E
    assert h.crc32c(bytes(range(31, -1, -1))) == 0x113FDB5C
    rng = np.random.RandomState(0)
    for n in (1, 7, 8, 9, 63, 4097):
        b = rng.bytes(n)
        assert h.crc32c(b) == h.crc32c_sw(b)                  # SSE4.2 == table
        assert h.crc32c_extend(h.crc32c(b[:3]), b[3:]) == h.crc32c(b)


def test_crc32c_mask(h):
    for c in (0, 1, 0xE3069283, 0xFFFFFFFF):
        assert h.crc32c_mask(c) == _mask_py(c)
        assert h.crc32c_unmask(h.crc32c_mask(c)) == c


# ---------------------------------------------------------------- bundle
def _write(h, prefix, tensors):
    h.write_bundle(prefix, [(n, dt, list(a.shape), a.tobytes()) for n, dt, a in tensors])


def test_bundle_roundtrip_and_layout(h, tmp_path):
    prefix = str(tmp_path / "model.ckpt-7")
    k = np.arange(12, dtype=np.float32).reshape(3, 4)
    b = np.array([1.5, -2.0], dtype=np.float32)
    s = np.array(7, dtype=np.int32)
    _write(h, prefix, [("global/dense/kernel", 1, k), ("global/global_step", 3, s),
                       ("global/dense/bias", 1, b)])
    assert sorted(os.listdir(tmp_path)) == ["model.ckpt-7.data-00000-of-00001",
                                            "model.ckpt-7.index"]
    out = h.read_bundle(prefix)
    assert np.frombuffer(out["global/dense/kernel"][2], np.float32).reshape(3, 4).tolist() == \
        k.tolist()
    assert out["global/global_step"][:2] == (3, [])
    # data file = tensors in sorted key order, no padding (BundleWriter default)
    data = open(prefix + ".data-00000-of-00001", "rb").read()
    assert data == b.tobytes() + k.tobytes() + s.tobytes()

    idx = open(prefix + ".index", "rb").read()
    # footer: magic of the LevelDB/TF table format
    assert struct.unpack("<Q", idx[-8:])[0] == 0xDB4775248B80FB57
    kv = h.read_table(idx)
    keys = [k_ for k_, _ in kv]
    assert keys == [b"", b"global/dense/bias", b"global/dense/kernel", b"global/global_step"]
    # BundleHeaderProto{num_shards: 1, version {producer: 1}}
    assert kv[0][1] == b"\x08\x01\x1a\x02\x08\x01"
    # BundleEntryProto of the kernel: dtype=1, shape {dim{3} dim{4}}, offset=8, size=48,
    # crc32c = masked crc of the bytes (fixed32, field 6)
    crc = _mask_py(h.crc32c(k.tobytes()))
    expect = (b"\x08\x01" + b"\x12\x08" + b"\x12\x02\x08\x03" + b"\x12\x02\x08\x04" +
              b"\x20\x08" + b"\x28\x30" + b"\x35" + struct.pack("<I", crc))
    assert kv[2][1] == expect
    # scalar shape: empty TensorShapeProto present
    assert kv[3][1].startswith(b"\x08\x03\x12\x00")


def test_bundle_detects_corruption(h, tmp_path):
    prefix = str(tmp_path / "c")
    _write(h, prefix, [("a", 1, np.ones(16, np.float32))])
    p = prefix + ".data-00000-of-00001"
    raw = bytearray(open(p, "rb").read())
    raw[5] ^= 0xFF
    open(p, "wb").write(bytes(raw))
    with pytest.raises(RuntimeError, match="checksum"):
        h.read_bundle(prefix)
    h.read_bundle(prefix, verify=False)


def test_table_many_keys_multiblock(h):
    kvs = [(b"key%06d" % i, os.urandom(300)) for i in range(2000)]  # > 256 KiB -> several blocks
    t = h.build_table(kvs)
    assert h.read_table(t) == kvs


# ---------------------------------------------------------------- events
def _frame_py(data, h):
    ln = struct.pack("<Q", len(data))
    return (ln + struct.pack("<I", _mask_py(h.crc32c(ln))) + data +
            struct.pack("<I", _mask_py(h.crc32c(data))))


def test_tfrecord_framing_and_event_protos(h, tmp_path):
    assert h.frame_record(b"abc") == _frame_py(b"abc", h)
    w = h.EventWriter(str(tmp_path), 100.0, "")
    w.add_scalars({"loss": 2.5}, 3, 1234.5)
    w.add_summary(h.summary_scalars({"accuracy": 0.75}), 4, 1235.0)
    w.add_scalar_series(["loss", "accuracy"], [5, 6], [[1.0, 0.5], [0.5, 1.0]], 1236.0)
    w.close()
    name = os.path.basename(w.path)
    assert name.startswith("events.out.tfevents.")
    recs = h.read_records(w.path)
    ev = [h.parse_event(r) for r in recs]
    assert ev[0]["file_version"] == "brain.Event:2"
    assert ev[1] == {"step": 3, "wall_time": 1234.5, "scalars": {"loss": 2.5}}
    assert ev[2]["scalars"] == {"accuracy": 0.75}
    assert [e["step"] for e in ev[3:]] == [5, 6]
    # Event{wall_time (fixed64, field 1), step (varint, 2), summary (5)}; Value{tag 1, simple 2}
    assert recs[1] == (b"\x09" + struct.pack("<d", 1234.5) + b"\x10\x03" + b"\x2a\x0d" +
                       b"\x0a\x0b\x0a\x04loss\x15" + struct.pack("<f", 2.5))


# ---------------------------------------------------------------- parameter server
@pytest.fixture
def ps(h):
    s = h.PSServer("127.0.0.1", 0)
    s.start()
    yield s
    s.stop()


def test_ps_protocol(h, ps):
    c = h.PSClient(["127.0.0.1:%d" % ps.port], 5.0)
    hw = c.create("global/w", "float32", [2, 3], 0)
    hs = c.create("global/global_step", "int64", [], 0)
    assert c.create("global/w", "float32", [2, 3], 0) == hw          # idempotent
    with pytest.raises(RuntimeError):
        c.create("global/w", "float32", [3, 3], 0)
    assert sorted(c.uninitialized([hw, hs])) == sorted([hw, hs])
    tmp = np.zeros(6, np.float32)
    with pytest.raises(RuntimeError, match="uninitialized"):
        c.pull([hw], [tmp.ctypes.data], [24])
    w = np.arange(6, dtype=np.float32)
    c.assign(hw, w.ctypes.data, 24)
    z = np.zeros(1, np.int64)
    c.assign(hs, z.ctypes.data, 8)
    assert c.uninitialized([hw, hs]) == []
    g = np.ones(6, np.float32)
    c.push_apply([hw], [g.ctypes.data], [24], 0.5)
    o = np.zeros(6, np.float32)
    c.pull([hw], [o.ctypes.data], [24])
    assert o.tolist() == (w - 0.5).tolist()
    assert [c.fetch_add(hs, 1) for _ in range(3)] == [0, 1, 2]
    assert c.lookup("global/w", 0) == hw
    with pytest.raises(RuntimeError):
        c.lookup("nope", 0)
    assert c.list_vars(0)[0] == ("global/w", "float32", [2, 3], True)


def test_ps_concurrent_workers(h, ps):
    """4 workers x 200 pushes: locked applies are exact; fetch_add is atomic."""
    addr = ["127.0.0.1:%d" % ps.port]
    c0 = h.PSClient(addr, 5.0)
    hw = c0.create("v", "float32", [1024], 0)
    hs = c0.create("s", "int64", [], 0)
    zw, zs = np.zeros(1024, np.float32), np.zeros(1, np.int64)  # keep alive across the call
    c0.assign(hw, zw.ctypes.data, 4096)
    c0.assign(hs, zs.ctypes.data, 8)
    seen = []

    def work():
        c = h.PSClient(addr, 5.0)
        g = np.ones(1024, np.float32)
        for _ in range(200):
            c.push_apply([hw], [g.ctypes.data], [4096], -1.0, True)
            seen.append(c.fetch_add(hs, 1))

    ts = [threading.Thread(target=work) for _ in range(4)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    o = np.zeros(1024, np.float32)
    c0.pull([hw], [o.ctypes.data], [4096])
    assert (o == 800).all()
    assert sorted(seen) == list(range(800))


def test_ps_sharding_two_tasks(h):
    servers = [h.PSServer("127.0.0.1", 0) for _ in range(2)]
    for s in servers:
        s.start()
    try:
        from distributedtensorflowexample_amd.parallel.ps import PSVariableStore

        specs = [("a", (4,), "float32"), ("b", (2,), "float32"), ("step", (), "int64")]
        st = PSVariableStore(["127.0.0.1:%d" % s.port for s in servers], specs).create()
        assert sorted(st.uninitialized()) == ["a", "b", "step"]
        st.assign({"a": np.ones(4), "b": np.full(2, 3.0), "step": 5})
        assert [s.num_vars() for s in servers] == [2, 1]  # round-robin a->0, b->1, step->0
        import torch

        st.push_apply({"a": torch.ones(4), "b": torch.ones(2)}, 0.5)
        v = st.read_all()
        assert v["a"].tolist() == [0.5] * 4 and v["b"].tolist() == [2.5, 2.5]
        assert int(v["step"]) == 5 and st.fetch_add("step") == 5
    finally:
        for s in servers:
            s.stop()


def test_ps_sync_replicas_rounds(h):
    """SYNC_PUSH (tf.train.SyncReplicasOptimizer semantics) over two ps tasks: 3 workers x 5
    rounds with R = 3 -- each round applies the MEAN of the 3 gradients once and advances
    global_step; a stale push (old local step) is dropped; an incomplete round times out."""
    import torch

    from distributedtensorflowexample_amd.parallel.ps import PSVariableStore

    servers = [h.PSServer("127.0.0.1", 0) for _ in range(2)]
    for s in servers:
        s.start()
    try:
        addrs = ["127.0.0.1:%d" % s.port for s in servers]
        specs = [("a", (64,), "float32"), ("b", (3,), "float32"),
                 ("global/global_step", (), "int64")]
        st0 = PSVariableStore(addrs, specs).create()
        st0.assign({"a": np.zeros(64), "b": np.zeros(3), "global/global_step": 7})
        results = {}

        def worker(k):
            st = PSVariableStore(addrs, specs).lookup()
            step = st.read_int("global/global_step")
            seq = []
            for _ in range(5):
                g = {"a": torch.full((64,), float(k + 1)), "b": torch.full((3,), 10.0 * (k + 1))}
                step, applied = st.sync_push(g, 0.5, 3, step, timeout_s=30)
                seq.append((step, applied))
            results[k] = seq
            st.close()

        ts = [threading.Thread(target=worker, args=(k,)) for k in range(3)]
        [t.start() for t in ts]
        [t.join() for t in ts]
        for k in range(3):  # every worker saw rounds 8..12, all applied
            assert results[k] == [(8 + i, True) for i in range(5)], results[k]
        v = st0.read_all()
        # mean gradient (1 + 2 + 3) / 3 = 2 per round for a, 20 for b: 5 rounds x 0.5 lr
        assert torch.allclose(v["a"], torch.full((64,), -5.0))
        assert torch.allclose(v["b"], torch.full((3,), -50.0))
        assert int(v["global/global_step"]) == 12
        assert sum(s.stats()["sync_rounds"] for s in servers) == 10  # 5 rounds on each task
        # a push tagged with an old step is dropped, not applied
        step, applied = st0.sync_push({"a": torch.ones(64), "b": torch.ones(3)}, 0.5, 3, 9)
        assert (step, applied) == (12, False)
        assert torch.allclose(st0.read_all()["a"], torch.full((64,), -5.0))
        # a round that never completes fails after its timeout instead of hanging
        with pytest.raises(RuntimeError, match="timed out"):
            st0.sync_push({"a": torch.ones(64), "b": torch.ones(3)}, 0.5, 3, 12, timeout_s=0.3)
        # ... and its gradient is withdrawn: retrying the same step (twice more, timing out
        # again) and then completing the round with two other replicas applies the mean of
        # exactly three gradients, the retry counted once
        with pytest.raises(RuntimeError, match="withdrawn"):
            st0.sync_push({"a": torch.ones(64), "b": torch.ones(3)}, 0.5, 3, 12, timeout_s=0.3)
        assert sum(s.stats()["sync_withdrawn"] for s in servers) == 4  # 2 pushes x 2 tasks
        outs = {}

        def push(k, val):
            st = PSVariableStore(addrs, specs).lookup()
            outs[k] = st.sync_push({"a": torch.full((64,), val), "b": torch.full((3,), val)},
                                   0.5, 3, 12, timeout_s=30)
            st.close()

        ts = [threading.Thread(target=push, args=(k, v)) for k, v in enumerate((1.0, 4.0, 7.0))]
        [t.start() for t in ts]
        [t.join() for t in ts]
        assert all(o == (13, True) for o in outs.values()), outs
        v = st0.read_all()
        assert torch.allclose(v["a"], torch.full((64,), -5.0 - 0.5 * 4.0))  # mean (1+4+7)/3
        st0.close()
    finally:
        for s in servers:
            s.stop()


def test_sync_replicas_optimizer_api(h, ps):
    """tf.train.SyncReplicasOptimizer-style wrapper: 2 replicas, R = 2, one averaged apply
    per step; R = 1 of 2 makes the slower replica a backup whose gradient is dropped."""
    import torch

    from distributedtensorflowexample_amd.optim import GradientDescentOptimizer
    from distributedtensorflowexample_amd.parallel.ps import PSVariableStore, SyncReplicasOptimizer

    addr = ["127.0.0.1:%d" % ps.port]
    specs = [("w", (8,), "float32"), ("global/global_step", (), "int64")]
    st = PSVariableStore(addr, specs).create()
    st.assign({"w": np.zeros(8), "global/global_step": 0})
    with pytest.raises(TypeError):
        SyncReplicasOptimizer(object(), 2, store=st)
    out = {}

    def replica(k, R):
        s = PSVariableStore(addr, specs).lookup()
        opt = SyncReplicasOptimizer(GradientDescentOptimizer(0.1), R, 2, store=s, timeout_s=20)
        steps = [opt.apply_gradients([(torch.full((8,), float(k + 1)), "w")]) for _ in range(3)]
        out[k] = (steps, opt.dropped)

    ts = [threading.Thread(target=replica, args=(k, 2)) for k in range(2)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert out[0][0] == out[1][0] == [1, 2, 3]
    assert torch.allclose(st.read_all()["w"], torch.full((8,), -0.1 * 1.5 * 3))
    # R = 1: the first push of a step applies alone; a push for an applied step is dropped
    opt = SyncReplicasOptimizer(GradientDescentOptimizer(0.1), 1, 2, store=st)
    assert opt.apply_gradients([(torch.ones(8), "w")]) == 4
    opt.local_step = 3  # a backup replica still on step 3
    assert opt.apply_gradients([(torch.ones(8), "w")]) == 4 and opt.dropped == 1


def test_ps_push_step_pull_one_round_trip(h):
    """push_step_pull: the pipelined push + fetch_add + pull over two ps tasks is served in
    the reference's order (apply, then step, then read): the pulled values include this
    push's update and the old step comes back."""
    import torch

    from distributedtensorflowexample_amd.parallel.ps import PSVariableStore

    servers = [h.PSServer("127.0.0.1", 0) for _ in range(2)]
    for s in servers:
        s.start()
    try:
        addrs = ["127.0.0.1:%d" % s.port for s in servers]
        specs = [("a", (1000,), "float32"), ("b", (7,), "float32"),
                 ("global/global_step", (), "int64")]
        st = PSVariableStore(addrs, specs).create()
        st.assign({"a": np.ones(1000), "b": np.full(7, 2.0), "global/global_step": 41})
        for k in range(3):
            old, vals = st.push_step_pull({"a": torch.full((1000,), 1.0),
                                           "b": torch.full((7,), 4.0)}, 0.25)
            assert old == 41 + k
            assert torch.allclose(vals["a"], torch.full((1000,), 1.0 - 0.25 * (k + 1)))
            assert torch.allclose(vals["b"], torch.full((7,), 2.0 - 1.0 * (k + 1)))
        assert st.read_int("global/global_step") == 44
        st.close()
    finally:
        for s in servers:
            s.stop()
