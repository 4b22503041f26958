"""Register budget of every built gfx950 kernel (CPU only: reads the code-object metadata
of the in-tree build, build/native/hip/*.hip.o).

No kernel may use scratch (private segment) or spill VGPRs: a spill in a hot kernel is a
silent 2-5x slowdown (docs/GEMM.md: a runtime-variant 256x256 GEMM fell from 1.1 to 0.2 PF
when it started spilling), so it is a test failure, not a perf note.  SGPR spills are
allowed only without scratch (they then live in VGPR lanes: v_writelane / v_readlane, no
memory traffic) -- e.g. the 8-rank xGMI kernels' 16 peer pointers."""
import glob
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
OBJS = sorted(glob.glob(os.path.join(ROOT, "build", "native", "hip", "*.hip.o")))

pytestmark = pytest.mark.skipif(not OBJS or not os.path.exists(os.path.join(LLVM, "llvm-readelf")),
                                reason="no in-tree HIP build or no ROCm LLVM tools")


def kernel_resources(obj):
    """[(kernel, private_segment_bytes, vgpr_spills, sgpr_spills, vgprs)] of the gfx950 code
    object embedded in a hipcc host object."""
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "k.hsaco")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section",
                        ".hip_fatbin=" + fb, obj], check=True, capture_output=True)
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--type=o", "--unbundle",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--input=" + fb,
                        "--output=" + co], check=True, capture_output=True)
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True,
                               capture_output=True, text=True).stdout
    out = []
    # one YAML map per kernel in the amdhsa.kernels list: split at each "- .agpr_count"/".args"
    for block in re.split(r"\n\s+- \.", notes):
        name = re.search(r"\n\s+\.name:\s+(\S+)", block)
        if not name:
            continue
        def num(key):
            m = re.search(r"\.%s:\s+(\d+)" % key, block)
            return int(m.group(1)) if m else 0
        out.append((name.group(1), num("private_segment_fixed_size"), num("vgpr_spill_count"),
                    num("sgpr_spill_count"), num("vgpr_count")))
    return out


@pytest.mark.parametrize("obj", OBJS, ids=[os.path.basename(o) for o in OBJS])
def test_no_scratch_no_spills(obj):
    ks = kernel_resources(obj)
    assert ks, "no kernels found in " + obj
    bad = [k for k in ks if k[1] or k[2]]
    assert not bad, "scratch / spills: " + "; ".join(
        "%s scratch=%dB vgpr_spill=%d sgpr_spill=%d" % (n[:90], s, v, g) for n, s, v, g, _ in bad)
