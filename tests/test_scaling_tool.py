"""tools/scaling.py: command construction and efficiency arithmetic (no GPU needed)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "tools"))

import scaling  # noqa: E402


def test_bench_command_shapes():
    c1 = scaling.bench_cmd(1, 100, 10, ["--model", "mlp"])
    assert c1[1].endswith("bench.py") and "--gpus" in c1 and "torch.distributed.run" not in c1
    c8 = scaling.bench_cmd(8, 100, 10, [])
    assert "torch.distributed.run" in c8 and c8[c8.index("--nproc-per-node") + 1] == "8"
    assert c8[c8.index("--master-addr") + 1] == "127.0.0.1"


def test_weak_scaling_efficiency():
    rs = [{"n_gpus": 1, "value": 100.0}, {"n_gpus": 2, "value": 180.0},
          {"n_gpus": 8, "value": 640.0}]
    out = scaling.efficiency(rs)
    assert [r["scaling_efficiency"] for r in out] == [1.0, 0.9, 0.8]
    assert scaling.efficiency([{"n_gpus": 2, "value": 1.0}])[0]["scaling_efficiency"] is None
