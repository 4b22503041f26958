"""Session/device configuration (``tf.GPUOptions`` / ``tf.ConfigProto``).

The reference shares one GPU between several worker processes by giving each
a memory fraction (main.py:58-64: ``0.9 / ceil(num_workers / num_gpus)``) and
sets ``allow_soft_placement`` for the session (worker.py:120-121).  Here the
fraction maps onto the PyTorch-ROCm caching allocator's per-process cap.
With 288 GB of HBM3E per MI355X the idiomatic layout is one process per GPU
(fraction 0.9), but multi-tenant PS workers are supported the same way.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field


@dataclass
class GPUOptions:
    per_process_gpu_memory_fraction: float = 0.0  # 0 = no cap
    allow_growth: bool = True
    visible_device_list: str = ""


@dataclass
class ConfigProto:
    gpu_options: GPUOptions = field(default_factory=GPUOptions)
    allow_soft_placement: bool = True
    log_device_placement: bool = False

    def apply(self, device=None):
        """Apply the memory cap to the current GPU (no-op without a GPU)."""
        frac = self.gpu_options.per_process_gpu_memory_fraction
        try:
            import torch

            if frac and torch.cuda.is_available():
                torch.cuda.set_per_process_memory_fraction(float(frac), device)
        except Exception:  # pragma: no cover - no device
            pass
        return self


def memory_fraction(num_workers, num_gpus, headroom=0.9):
    """main.py:58-60: 0.9 / ceil(num_workers / num_gpus)."""
    return headroom / math.ceil(float(num_workers) / float(max(1, num_gpus)))


_HIP_SCHED = {"auto": 0, "spin": 1, "yield": 2, "blocking": 4}


def apply_hip_schedule(mode=None):
    """How this process's host threads wait for the GPU (``hipSetDeviceFlags``): ``spin``,
    ``yield``, ``blocking`` (sleep on an interrupt) or ``auto`` (the runtime's choice).  Several
    async-PS workers share one host's CPU share with the ps threads, and spinning waiters take
    cycles from them.  ``mode`` None reads ``DTFX_HIP_SCHED``; unset: leave the default.  Must run
    before the process touches the GPU.  Returns the flag value set, or None."""
    mode = mode if mode is not None else os.environ.get("DTFX_HIP_SCHED")
    if not mode:
        return None
    if mode not in _HIP_SCHED:
        raise ValueError("DTFX_HIP_SCHED must be one of %s" % sorted(_HIP_SCHED))
    import ctypes

    import torch

    lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    rc = lib.hipSetDeviceFlags(ctypes.c_uint(_HIP_SCHED[mode]))
    if rc != 0:
        raise RuntimeError("hipSetDeviceFlags(%s) failed: %d" % (mode, rc))
    return _HIP_SCHED[mode]
