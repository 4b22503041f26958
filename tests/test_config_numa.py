"""Host placement helpers of the async-PS cluster (config.py, --cpu_affinity numa): sysfs
parsing against a fake tree, the ps / worker core slots, affinity pinning (CPU only)."""
import os

import pytest

from distributedtensorflowexample_amd import config


def _write(path, text):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        f.write(text)


def test_numa_nodes_parses_cpulists(tmp_path):
    _write(str(tmp_path / "node0" / "cpulist"), "0-3,8-11\n")
    _write(str(tmp_path / "node1" / "cpulist"), "4-7\n")
    _write(str(tmp_path / "possible"), "0-1\n")  # not a node directory
    assert config.numa_nodes(str(tmp_path)) == {0: [0, 1, 2, 3, 8, 9, 10, 11], 1: [4, 5, 6, 7]}
    assert config.numa_nodes(str(tmp_path / "missing")) == {}


def test_first_gpu_numa_node_from_kfd_topology(tmp_path):
    topo, pci = tmp_path / "topo", tmp_path / "pci"
    # node 0: a CPU agent (no SIMDs); node 1: the first GPU at 0000:75:00.0
    _write(str(topo / "0" / "properties"), "cpu_cores_count 64\nsimd_count 0\n")
    loc = (0x75 << 8) | (0 << 3) | 0
    _write(str(topo / "1" / "properties"), "simd_count 1024\nlocation_id %d\ndomain 0\n" % loc)
    _write(str(pci / "0000:75:00.0" / "numa_node"), "1\n")
    assert config.first_gpu_numa_node_sysfs(str(topo), str(pci)) == 1
    # a second GPU (node 2 of the topology) on the other socket: index 1
    loc2 = (0xf5 << 8)
    _write(str(topo / "2" / "properties"), "simd_count 1024\nlocation_id %d\ndomain 0\n" % loc2)
    _write(str(pci / "0000:f5:00.0" / "numa_node"), "0\n")
    assert config.first_gpu_numa_node_sysfs(str(topo), str(pci), index=1) == 0
    assert config.first_gpu_numa_node_sysfs(str(topo), str(pci), index=2) is None
    _write(str(pci / "0000:75:00.0" / "numa_node"), "-1\n")  # firmware says nothing
    assert config.first_gpu_numa_node_sysfs(str(topo), str(pci)) is None
    assert config.first_gpu_numa_node_sysfs(str(tmp_path / "none"), str(pci)) is None


def test_visible_gpu_index():
    assert config.visible_gpu_index({}) == 0
    assert config.visible_gpu_index({"HIP_VISIBLE_DEVICES": "3"}) == 3
    assert config.visible_gpu_index({"HIP_VISIBLE_DEVICES": "5,6"}) == 5
    assert config.visible_gpu_index({"HIP_VISIBLE_DEVICES": "", "CUDA_VISIBLE_DEVICES": "2"}) == 2
    assert config.visible_gpu_index({"HIP_VISIBLE_DEVICES": "GPU-1234abcd"}) == 0


def test_cpu_slots_do_not_overlap():
    for num_ps in (1, 2):
        used = set()
        for t in range(num_ps):
            n, off = config.ps_cpu_slot(t)
            s = set(range(off, off + n))
            assert not s & used
            used |= s
        for i in range(16):
            n, off = config.worker_cpu_slot(i, num_ps)
            s = set(range(off, off + n))
            assert not s & used, (num_ps, i)
            used |= s


def test_pin_to_numa_node(monkeypatch):
    monkeypatch.setattr(config, "numa_nodes", lambda: {0: [0, 1, 2, 3], 1: [4, 5, 6, 7]})
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: {0, 1, 2, 3, 4, 5, 6})
    got = []
    monkeypatch.setattr(os, "sched_setaffinity", lambda pid, cpus: got.append(list(cpus)))
    assert config.pin_to_numa_node(1) == [4, 5, 6]        # allowed CPUs of the node only
    assert config.pin_to_numa_node(0, count=2, offset=2) == [2, 3]  # a slot inside the node
    assert config.pin_to_numa_node(0, count=2, offset=3) is None    # would wrap: not pinned
    assert config.pin_to_numa_node(None) is None
    assert config.pin_to_numa_node(5) is None            # unknown node: left alone
    assert got == [[4, 5, 6], [2, 3]]


def test_hip_schedule_modes(monkeypatch):
    monkeypatch.delenv("DTFX_HIP_SCHED", raising=False)
    assert config.apply_hip_schedule() is None          # unset: the runtime's default
    with pytest.raises(ValueError):
        config.apply_hip_schedule("busy")
