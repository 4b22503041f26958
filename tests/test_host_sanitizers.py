"""Host C++ runtime (PS server/client, TF-V2 bundle, event writer, CRC32C) under
AddressSanitizer + UBSan and ThreadSanitizer, via tools/sanitize_host.py:
an instrumented build of csrc/host driven by a multi-threaded self-test in a child
interpreter.  CPU only."""
import os
import shutil
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "tools"))
import sanitize_host  # noqa: E402

pytestmark = pytest.mark.skipif(shutil.which(sanitize_host._cxx()) is None, reason="no g++")


@pytest.mark.timeout(900)
def test_host_runtime_clean_under_asan_ubsan():
    rc, out = sanitize_host.run("asan")
    assert rc == 0 and "host selftest ok" in out, out[-6000:]


@pytest.mark.timeout(900)
def test_host_runtime_clean_under_tsan_and_detector_live():
    rc, out = sanitize_host.run("tsan")
    assert rc == 0 and "host selftest ok" in out, out[-6000:]
    # without the two suppressions the reference's intentional Hogwild / lock-free-pull
    # races are reported: the detector is active, and those are the only races
    rc, out = sanitize_host.run("tsan", suppress=False, rebuild=False)
    assert rc != 0 and "ThreadSanitizer: data race" in out, out[-3000:]
    assert "dtfx_hogwild_apply" in out or "dtfx_racy_read" in out, out[-6000:]
