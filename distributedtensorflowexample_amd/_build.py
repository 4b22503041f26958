"""In-tree native build: hipcc for the gfx950 kernels, g++ for the host runtime.

Two extension modules are produced next to this file:

* ``_hip``  -- every ``csrc/kernels/*.hip`` compiled with
  ``hipcc --offload-arch=gfx950`` plus the pybind11 launcher bindings.
* ``_host`` -- the host-side C++ runtime (``csrc/host/*.cpp``): CRC32C,
  TF-V2 tensor-bundle checkpoints, TFRecord event files, the TCP parameter
  server and the IDX reader.

The build is incremental (object newer than its source and every header =>
skipped) and parallel.  No torch cpp_extension / hipify step is involved: the
kernels are written for CDNA4 directly and the bindings take raw device
addresses, so nothing is translated.

Usage::

    python -m distributedtensorflowexample_amd._build          # both modules
    python -m distributedtensorflowexample_amd._build --only host
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
ARCH = os.environ.get("DTFX_OFFLOAD_ARCH", "gfx950")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _pybind_includes():
    import pybind11

    return [pybind11.get_include(), sysconfig.get_paths()["include"]]


def _torch_lib_dir():
    """Directory of the HIP runtime torch ships (same SONAME as /opt/rocm's).

    Linking against it and putting it first on the rpath keeps ONE HIP runtime
    in the process however the modules are imported.
    """
    try:
        import importlib.util

        spec = importlib.util.find_spec("torch")
        if spec and spec.origin:
            d = os.path.join(os.path.dirname(spec.origin), "lib")
            if os.path.exists(os.path.join(d, "libamdhip64.so")):
                return d
    except Exception:
        pass
    return None


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm 7.x expected at /opt/rocm)")


def _newer(target, deps):
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(d) <= t for d in deps if os.path.exists(d))


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build step failed:\n  %s\n%s" % (" ".join(cmd), r.stdout))
    return r.stdout


def _compile_all(jobs, verbose):
    with cf.ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        futs = {ex.submit(_run, cmd): out for cmd, out in jobs}
        for f in cf.as_completed(futs):
            out = f.result()
            if verbose and out.strip():
                print(out)


def build_hip(verbose=False, force=False):
    src_dir = os.path.join(CSRC, "kernels")
    obj_dir = os.path.join(BUILD, "hip")
    os.makedirs(obj_dir, exist_ok=True)
    headers = glob.glob(os.path.join(src_dir, "*.h"))
    hipcc = _hipcc()
    common = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-Wno-unused-result"]
    jobs, objs = [], []
    for src in sorted(glob.glob(os.path.join(src_dir, "*.hip"))):
        obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or not _newer(obj, [src] + headers):
            jobs.append(([hipcc, "-c", "-x", "hip", src, "-o", obj] + common, obj))
    inc = sum([["-I", d] for d in _pybind_includes()], [])
    for cpp in sorted(glob.glob(os.path.join(src_dir, "*.cpp"))):  # host-side C++ (bindings, RCCL)
        obj = os.path.join(obj_dir, os.path.basename(cpp) + ".o")
        objs.append(obj)
        if force or not _newer(obj, [cpp] + headers):
            jobs.append(([hipcc, "-c", cpp, "-o", obj, "-O2", "-std=c++17", "-fPIC",
                          "-fvisibility=hidden", "-D__HIP_PLATFORM_AMD__"] + inc, obj))
    _compile_all(jobs, verbose)
    out = os.path.join(PKG_DIR, "_hip" + EXT_SUFFIX)
    if force or jobs or not _newer(out, objs):
        link = [hipcc, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", out] + objs
        tl = _torch_lib_dir()
        if tl:
            link += ["-L" + tl, "-Wl,-rpath," + tl]
        link += ["-lamdhip64", "-lrccl"]
        _run(link)
    return out


def build_host(verbose=False, force=False):
    src_dir = os.path.join(CSRC, "host")
    obj_dir = os.path.join(BUILD, "host")
    os.makedirs(obj_dir, exist_ok=True)
    headers = glob.glob(os.path.join(src_dir, "*.h"))
    cxx = os.environ.get("CXX", "g++")
    inc = sum([["-I", d] for d in _pybind_includes()], [])
    flags = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-msse4.2", "-pthread",
             "-Wall", "-Wno-unused-function"]
    jobs, objs = [], []
    for src in sorted(glob.glob(os.path.join(src_dir, "*.cpp"))):
        obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or not _newer(obj, [src] + headers):
            jobs.append(([cxx, "-c", src, "-o", obj] + flags + inc, obj))
    _compile_all(jobs, verbose)
    out = os.path.join(PKG_DIR, "_host" + EXT_SUFFIX)
    if force or jobs or not _newer(out, objs):
        _run([cxx, "-shared", "-o", out] + objs + ["-pthread"])
    return out


def build(only=None, verbose=False, force=False):
    outs = []
    if only in (None, "host"):
        outs.append(build_host(verbose, force))
    if only in (None, "hip"):
        outs.append(build_hip(verbose, force))
    return outs


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", choices=["hip", "host"], default=None)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    for o in build(a.only, a.verbose, a.force):
        print("built", os.path.relpath(o, ROOT))


if __name__ == "__main__":
    sys.exit(main())
