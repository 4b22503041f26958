"""Host C++ runtime under sanitizers (race detection / sanitizers).

Builds ``csrc/host/*.cpp`` (CRC32C, TF-V2 tensor bundle, TFRecord event writer with its
flush thread, TCP parameter server + client) as a separate ``_host`` module instrumented
with

* ``asan``: AddressSanitizer + UndefinedBehaviorSanitizer (``-fsanitize=address,undefined``)
* ``tsan``: ThreadSanitizer (``-fsanitize=thread``)

into ``build/sanitize/<kind>/`` and runs a self-test in a CHILD interpreter with the
sanitizer runtime preloaded (Python itself is not instrumented).  The self-test drives
every native entry point, including 4 client threads x (pull, locked push, fetch_add)
against one server, concurrent event-writer calls and a server stop with live
connections.  Any sanitizer report fails the run (``halt_on_error=1``, non-zero exit).

The reference's two INTENTIONAL races -- lock-free pulls and Hogwild applies
(worker.py:79, ``ApplyGradientDescent(use_locking=False)``) -- live only in
``dtfx_racy_read`` / ``dtfx_hogwild_apply`` (csrc/host/ps.cpp) and are the only TSan
suppressions.  Host code only: GPU sanitizers are not used on this hardware pool.

    python tools/sanitize_host.py [--kinds asan tsan]
"""
from __future__ import annotations

import argparse
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "csrc", "host")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
FLAGS = {
    "asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
    "tsan": ["-fsanitize=thread"],
}
RUNTIME = {"asan": "libasan.so", "tsan": "libtsan.so", "stdcxx": "libstdc++.so"}
TSAN_SUPPRESSIONS = "race:dtfx_racy_read\nrace:dtfx_hogwild_apply\n"


def _cxx():
    return os.environ.get("CXX", "g++")


def build(kind, out_dir=None):
    """Compile + link the instrumented module; returns its directory."""
    import pybind11

    out_dir = out_dir or os.path.join(ROOT, "build", "sanitize", kind)
    os.makedirs(out_dir, exist_ok=True)
    inc = ["-I", pybind11.get_include(), "-I", sysconfig.get_paths()["include"]]
    base = ["-O1", "-g", "-fno-omit-frame-pointer", "-std=c++17", "-fPIC", "-msse4.2",
            "-pthread"] + FLAGS[kind]
    procs, objs = [], []
    for src in sorted(glob.glob(os.path.join(SRC, "*.cpp"))):
        obj = os.path.join(out_dir, os.path.basename(src) + ".o")
        objs.append(obj)
        procs.append(subprocess.Popen([_cxx(), "-c", src, "-o", obj] + base + inc,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    for p in procs:
        out = p.communicate()[0]
        if p.returncode:
            raise RuntimeError("sanitizer build failed:\n" + out.decode(errors="replace"))
    so = os.path.join(out_dir, "_host" + EXT)
    subprocess.run([_cxx(), "-shared", "-o", so] + objs + base, check=True)
    return out_dir


def runtime_path(kind):
    p = subprocess.run([_cxx(), "-print-file-name=" + RUNTIME[kind]], capture_output=True,
                       text=True, check=True).stdout.strip()
    if not os.path.isabs(p) or not os.path.exists(p):
        raise RuntimeError("%s runtime not found (%s)" % (kind, p))
    return p


def run(kind, timeout=600, suppress=True, rebuild=True):
    """Build, then run the self-test under ``kind``; returns (returncode, output).
    ``suppress=False`` (tsan): no suppressions -- the intentional Hogwild race must then be
    reported (a check that the detector is live)."""
    mod_dir = build(kind) if rebuild else os.path.join(ROOT, "build", "sanitize", kind)
    env = dict(os.environ)
    # libstdc++ preloaded too: the sanitizer's __cxa_throw interceptor needs it resolvable
    # at startup (python does not link it)
    env["LD_PRELOAD"] = runtime_path(kind) + " " + runtime_path("stdcxx")
    env["PYTHONPATH"] = mod_dir
    env["ASAN_OPTIONS"] = "detect_leaks=0:halt_on_error=1:abort_on_error=0:exitcode=66"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    if kind == "tsan":
        sup = os.path.join(mod_dir, "tsan.supp")
        with open(sup, "w") as f:
            f.write(TSAN_SUPPRESSIONS if suppress else "")
        env["TSAN_OPTIONS"] = "halt_on_error=1:exitcode=66:suppressions=" + sup
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--selftest"], env=env,
                       capture_output=True, text=True, timeout=timeout, cwd=mod_dir)
    return r.returncode, r.stdout + r.stderr


# ---------------------------------------------------------------- self-test (child)
def selftest():
    import tempfile
    import threading

    import numpy as np

    import _host as h  # the instrumented module (PYTHONPATH)

    assert "sanitize" in h.__file__, h.__file__
    # CRC32C (hardware + table paths)
    rng = np.random.RandomState(0)
    for n in (0, 1, 7, 8, 9, 63, 4097):
        b = rng.bytes(n)
        assert h.crc32c(b) == h.crc32c_sw(b)
    assert h.crc32c(b"123456789") == 0xE3069283
    with tempfile.TemporaryDirectory() as d:
        # TF-V2 bundle round trip + corruption detection
        prefix = os.path.join(d, "model.ckpt-1")
        k = np.arange(12, dtype=np.float32).reshape(3, 4)
        h.write_bundle(prefix, [("global/dense/kernel", 1, [3, 4], k.tobytes()),
                                ("global/global_step", 9, [], np.int64(5).tobytes())])
        out = h.read_bundle(prefix)
        assert np.frombuffer(out["global/dense/kernel"][2], np.float32).tolist() == \
            k.ravel().tolist()
        kvs = [(b"key%06d" % i, rng.bytes(300)) for i in range(1500)]
        assert h.read_table(h.build_table(kvs)) == kvs
        raw = bytearray(open(prefix + ".data-00000-of-00001", "rb").read())
        raw[3] ^= 0xFF
        open(prefix + ".data-00000-of-00001", "wb").write(bytes(raw))
        try:
            h.read_bundle(prefix)
            raise AssertionError("corruption not detected")
        except RuntimeError:
            pass
        # event writer: its flush thread vs concurrent writers
        w = h.EventWriter(d, 0.01, "")
        evs = []

        def writer(t):
            for s in range(200):
                w.add_scalars({"loss%d" % t: float(s)}, s, 1000.0 + s)
            evs.append(t)

        ts = [threading.Thread(target=writer, args=(t,)) for t in range(3)]
        [t.start() for t in ts]
        for _ in range(5):
            w.flush()
        [t.join() for t in ts]
        w.close()
        recs = h.read_records(w.path)
        assert len(recs) == 1 + 3 * 200, len(recs)
        for r in recs[1:5]:
            h.parse_event(r)

    # parameter server: 4 client threads (pull, locked push, fetch_add), then a stop with
    # connections still open
    srv = h.PSServer("127.0.0.1", 0)
    srv.start()
    addr = ["127.0.0.1:%d" % srv.port]
    c0 = h.PSClient(addr, 5.0)
    hw = c0.create("w", "float32", [4096], 0)
    hs = c0.create("step", "int64", [], 0)
    zw, zs = np.zeros(4096, np.float32), np.zeros(1, np.int64)
    c0.assign(hw, zw.ctypes.data, zw.nbytes)
    c0.assign(hs, zs.ctypes.data, zs.nbytes)
    seen, errs = [], []
    clients = []

    def work(i):
        try:
            c = h.PSClient(addr, 5.0)
            clients.append(c)
            g = np.ones(4096, np.float32)
            buf = np.empty(4096, np.float32)
            for it in range(100):
                c.pull([hw], [buf.ctypes.data], [buf.nbytes])
                c.push_apply([hw], [g.ctypes.data], [g.nbytes], -1.0, it % 2 == 0)
                seen.append(c.fetch_add(hs, 1))
            try:
                c.pull([hw + (7 << 32)], [buf.ctypes.data], [buf.nbytes])  # unknown task
                errs.append("bad handle accepted")
            except RuntimeError:
                pass
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    ts = [threading.Thread(target=work, args=(i,)) for i in range(4)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errs, errs
    assert sorted(seen) == list(range(400))
    o = np.empty(4096, np.float32)
    c0.pull([hw], [o.ctypes.data], [o.nbytes])
    assert o.min() >= 1 and o.max() <= 400  # Hogwild pushes may be lost, never invented
    assert [v[0] for v in c0.list_vars(0)] == ["w", "step"]
    # split-phase exchange (push + step + pull in flight) closed from ANOTHER thread: close()
    # runs without the GIL and waits for the owner's end(), which needs the GIL (round-5 fix)
    g1, b1 = np.ones(4096, np.float32), np.empty(4096, np.float32)
    args = ([hw], [g1.ctypes.data], [g1.nbytes], -1.0, False, hs, 1, [hw], [b1.ctypes.data],
            [b1.nbytes])
    c1 = h.PSClient(addr, 5.0)
    c1.push_step_pull_begin(*args)
    closer = threading.Thread(target=c1.close)
    closer.start()
    c1.push_step_pull_end()
    closer.join(10.0)
    assert not closer.is_alive(), "close() deadlocked against an open exchange"
    # a client dropped with its exchange still open: the destructor must not wait for end()
    c2 = h.PSClient(addr, 5.0)
    c2.push_step_pull_begin(*args)
    del c2
    srv.stop()  # clients still connected
    for c in clients + [c0]:
        c.close()
    print("host selftest ok")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kinds", nargs="+", default=["asan", "tsan"], choices=list(FLAGS))
    ap.add_argument("--selftest", action="store_true", help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.selftest:
        selftest()
        return 0
    rc_all = 0
    for kind in a.kinds:
        rc, out = run(kind)
        print("== %s: rc %d" % (kind, rc))
        print(out[-4000:] if rc == 0 else out[-20000:])
        rc_all = rc_all or rc
    return rc_all


if __name__ == "__main__":
    sys.exit(main())
