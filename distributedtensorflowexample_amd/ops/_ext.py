"""Loader for the native extension modules.

``hip()`` returns the gfx950 kernel module (``_hip``) and raises loudly when
it is missing or was built for another arch: a GPU tensor never silently
falls back to a PyTorch implementation.  CPU tensors take the explicit CPU
reference path of each op (used by the CPU test tier and the CPU-only
parameter-server "plumbing" configuration of BASELINE.json).
"""
from __future__ import annotations

import importlib

import torch

_HIP = None
_HIP_ERR = None
_HOST = None
_HOST_ERR = None


def hip():
    global _HIP, _HIP_ERR
    if _HIP is None and _HIP_ERR is None:
        try:
            _HIP = importlib.import_module("distributedtensorflowexample_amd._hip")
        except Exception as e:  # pragma: no cover - depends on build state
            _HIP_ERR = e
    if _HIP is None:
        raise RuntimeError(
            "distributedtensorflowexample_amd._hip (gfx950 kernels) is not built or failed "
            "to load: %r. Run `python -m distributedtensorflowexample_amd._build`." % (_HIP_ERR,))
    return _HIP


def host():
    global _HOST, _HOST_ERR
    if _HOST is None and _HOST_ERR is None:
        try:
            _HOST = importlib.import_module("distributedtensorflowexample_amd._host")
        except Exception as e:  # pragma: no cover
            _HOST_ERR = e
    if _HOST is None:
        raise RuntimeError(
            "distributedtensorflowexample_amd._host (native host runtime) is not built or "
            "failed to load: %r. Run `python -m distributedtensorflowexample_amd._build`."
            % (_HOST_ERR,))
    return _HOST


def hip_available() -> bool:
    try:
        hip()
        return True
    except RuntimeError:
        return False


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_cur_device = getattr(torch._C, "_cuda_getDevice", None)


def stream_handle(device=None) -> int:
    """Raw hipStream_t of the current torch stream (capture-aware: under graph capture it is
    the capture stream).  Read through the raw-stream accessor -- no Python ``Stream`` object
    per call (~2-3 us of host time ahead of every eager launch, which a driver-sized MLP
    region of 20 steps pays before its first kernel)."""
    if _raw_stream is None or _cur_device is None:
        return torch.cuda.current_stream(device).cuda_stream
    if device is None:
        idx = _cur_device()
    elif isinstance(device, int):
        idx = device
    else:
        idx = torch.device(device).index
        if idx is None:
            idx = _cur_device()
    return _raw_stream(idx)


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def check_gpu_f32(*ts, contiguous=True):
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise ValueError("expected a GPU tensor")
        if t.dtype != torch.float32:
            raise TypeError("expected float32, got %s" % t.dtype)
        if contiguous and not t.is_contiguous():
            raise ValueError("expected a contiguous tensor")
