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


# ---------------------------------------------------------------------------------------------
# NUMA placement of the async-PS cluster's host processes (--cpu_affinity numa).  Measured
# (tools/probes/ps_capacity.py, 2-socket box, profiles/r5/ps/): the ps alone served 8 clients
# at 5.9K round trips/s with its threads free to roam both sockets, 64K in the compact layout
# below; the whole cluster at 8 workers 0.88 M -> 1.49-1.52 M samples/s.


def numa_nodes(base="/sys/devices/system/node"):
    """{node: [cpu, ...]} from sysfs ({} where it says nothing)."""
    out = {}
    try:
        names = os.listdir(base)
    except OSError:
        return out
    for d in names:
        if not (d.startswith("node") and d[4:].isdigit()):
            continue
        try:
            cl = open(os.path.join(base, d, "cpulist")).read().strip()
        except OSError:
            continue
        cpus = []
        for part in cl.split(","):
            if not part:
                continue
            lo, _, hi = part.partition("-")
            cpus.extend(range(int(lo), int(hi or lo) + 1))
        out[int(d[4:])] = cpus
    return out


def _pci_numa_node(domain, bus, dev, fn=0, pci="/sys/bus/pci/devices"):
    try:
        n = int(open(os.path.join(pci, "%04x:%02x:%02x.%x" % (domain, bus, dev, fn),
                                  "numa_node")).read())
        return n if n >= 0 else None
    except (OSError, ValueError):
        return None


def gpu_numa_node(device_index=0):
    """NUMA node of a visible GPU (the worker process, which uses the GPU anyway)."""
    try:
        import torch

        p = torch.cuda.get_device_properties(device_index)
        return _pci_numa_node(p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
    except Exception:  # noqa: BLE001 - best effort
        return None


def first_gpu_numa_node_sysfs(base="/sys/class/kfd/kfd/topology/nodes",
                              pci="/sys/bus/pci/devices", index=0):
    """Node of the ``index``-th GPU of the KFD topology (the physical device numbering that
    ``HIP_VISIBLE_DEVICES`` selects from), without touching the GPU: the ps process, and a
    worker before its first GPU call (so the runtime's threads inherit the placement)."""
    try:
        nodes = sorted(os.listdir(base), key=lambda v: int(v) if v.isdigit() else 1 << 30)
    except OSError:
        return None
    for n in nodes:
        try:
            props = dict(l.split() for l in open(os.path.join(base, n, "properties"))
                         if len(l.split()) == 2)
        except (OSError, ValueError):
            continue
        if int(props.get("simd_count", "0")) <= 0:
            continue
        if index > 0:
            index -= 1
            continue
        loc, dom = int(props.get("location_id", "0")), int(props.get("domain", "0"))
        return _pci_numa_node(dom, loc >> 8, (loc >> 3) & 31, loc & 7, pci=pci)
    return None


def visible_gpu_index(env=None):
    """Physical index of the first GPU this process is given (``HIP_VISIBLE_DEVICES`` /
    ``CUDA_VISIBLE_DEVICES``, as the launcher sets them per worker), 0 when unset or not a
    plain index (UUIDs, empty)."""
    env = os.environ if env is None else env
    for k in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(k, "").split(",")[0].strip()
        if v.isdigit():
            return int(v)
    return 0


def pin_to_numa_node(node, count=0, offset=0):
    """Restrict the calling thread -- and every thread it starts afterwards, so call it before
    the first GPU call (the HIP runtime's threads) -- to allowed CPUs of ``node``: all of them
    (``count`` 0), or the ``count`` CPUs at positions ``offset`` .. ``offset + count - 1`` of
    the node's sorted list.  A slot that does not fit on the node (a small node or cpuset: it
    would wrap onto another process's cores, e.g. a worker onto the ps cores) is not pinned:
    a warning, and the placement is left to the scheduler.  Returns the CPU list, or None
    (unknown node / nothing allowed there / slot does not fit: left as it was)."""
    if node is None:
        return None
    allowed = os.sched_getaffinity(0)
    cpus = [c for c in sorted(numa_nodes().get(int(node), [])) if c in allowed]
    if not cpus:
        return None
    if count > 0:
        if offset + count > len(cpus):
            import sys

            print("[affinity] NUMA node %d has %d usable CPUs; slot %d..%d does not fit: not "
                  "pinned (--cpu_affinity none placement)" % (int(node), len(cpus), offset,
                                                              offset + count - 1),
                  file=sys.stderr, flush=True)
            return None
        cpus = cpus[offset:offset + count]
    os.sched_setaffinity(0, cpus)
    return cpus


# --cpu_affinity numa layout: ps task t on 8 consecutive cores (one shared-L3 core complex on
# the EPYC hosts of this pool) of GPU 0's node; worker i on 2 cores of ITS GPU's node, at the
# offset after the ps tasks' cores (the same positions are left free on every node, so a worker
# on GPU 0's node never lands on a ps core) -- instead of spread by the scheduler over 256 CPUs
PS_CPUS, WORKER_CPUS = 8, 2


def ps_cpu_slot(task_index):
    return PS_CPUS, PS_CPUS * int(task_index)


def worker_cpu_slot(task_index, num_ps):
    return WORKER_CPUS, PS_CPUS * int(num_ps) + WORKER_CPUS * int(task_index)
