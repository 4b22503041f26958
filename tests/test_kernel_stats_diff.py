"""tools/kernel_stats_diff.py: per-step kernel time difference of two rocprofv3 --stats CSVs,
steps given as a number or as the call count of a once-per-step kernel (k=<substring>)."""
import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _csv(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Name", "Calls", "TotalDurationNs"])
        w.writeheader()
        for name, calls, ns in rows:
            w.writerow({"Name": name, "Calls": calls, "TotalDurationNs": ns})


def test_diff_per_step(tmp_path):
    a, b = str(tmp_path / "a.csv"), str(tmp_path / "b.csv")
    _csv(a, [("gemm", 40, 40000), ("adam_kernel", 10, 5000)])             # 10 steps
    _csv(b, [("gemm", 20, 30000), ("adam_kernel", 5, 2500), ("allreduce", 5, 10000)])  # 5 steps
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "kernel_stats_diff.py"),
                          a, "k=adam", b, "k=adam"], capture_output=True, text=True, check=True)
    lines = out.stdout.splitlines()
    assert "10 steps" in lines[0] and "5 steps" in lines[1]
    body = {l.split()[-1]: [float(v) for v in l.split()[:3]] for l in lines[3:]
            if not l.strip().endswith("step")}
    assert body["allreduce"] == [0.0, 2.0, 2.0]      # us per step
    assert body["gemm"] == [4.0, 6.0, 2.0]
    assert body["adam_kernel"] == [0.5, 0.5, 0.0]
    assert lines[-1].split()[:3] == ["4.5", "8.5", "+4.0"]
