"""Where the driver-sized MLP region's fixed cost goes, on the GPU's own clock: run the bench's
timed region (synchronize; t0; run_launched(K, flush=True); synchronize; t1) REPS times under
``rocprofv3 --kernel-trace`` and line the host clock up with the kernel trace (both
CLOCK_MONOTONIC ns).  A tiny fill kernel before each region marks it in the trace.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/probes/k20_trace.py
    python3 tools/probes/k20_trace.py --analyze OUT/run_kernel_trace.csv OUT/k20_host.json

Per region: host t0 -> first kernel start (launch latency), the K steps' kernel durations and
the gaps between dependent kernels, the flush kernel, last kernel end -> host t1 (completion
wake-up), medians over the regions.
"""
import argparse
import csv
import json
import os
import sys
import time


def run(out, K, reps):
    import torch

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from distributedtensorflowexample_amd.data.synthetic import mnist_like_device
    from distributedtensorflowexample_amd.models.mlp import init_params
    from distributedtensorflowexample_amd.train.fused_mlp import FusedMLPTrainer

    dev = torch.device("cuda:0")
    x, y = mnist_like_device(55000, seed=100, device=dev)
    tr = FusedMLPTrainer(init_params(dev, seed=1234), x, y)
    tr.run(5)
    tr.run_launched(50)
    tr.flush()
    mark = torch.zeros(64, device=dev)
    regions = []
    for _ in range(reps):
        tr.run_launched(1)  # an update pending, as in the bench
        mark.fill_(1.0)     # the marker kernel
        torch.cuda.synchronize()
        time.sleep(0.0005)  # the bench's gap between the last untimed work and the clock
        torch.cuda.synchronize()
        t0 = time.monotonic_ns()
        tr.run_launched(K, flush=True)
        torch.cuda.synchronize()
        t1 = time.monotonic_ns()
        regions.append({"t0": t0, "t1": t1})
    json.dump({"K": K, "regions": regions}, open(out, "w"))
    print(json.dumps({"K": K, "wall_us": sorted((r["t1"] - r["t0"]) / 1e3 for r in regions)}))


def med(v):
    v = sorted(v)
    return round(v[len(v) // 2], 2) if v else None


def analyze(trace, host):
    h = json.load(open(host))
    K = h["K"]
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                for r in csv.DictReader(open(trace)))
    rows = []
    for reg in h["regions"]:
        inside = [k for k in ks if reg["t0"] <= k[0] <= reg["t1"]]
        if len(inside) != 2 * K + 1:
            continue
        d = [(e - s) / 1e3 for s, e, _ in inside]
        gaps = [(inside[i + 1][0] - inside[i][1]) / 1e3 for i in range(len(inside) - 1)]
        rows.append({
            "wall_us": (reg["t1"] - reg["t0"]) / 1e3,
            "host_t0_to_first_kernel_us": (inside[0][0] - reg["t0"]) / 1e3,
            "last_kernel_end_to_host_t1_us": (reg["t1"] - inside[-1][1]) / 1e3,
            "gpu_span_us": (inside[-1][1] - inside[0][0]) / 1e3,
            "first_launch_us_step1": d[0], "head_us_step1": d[1],
            "first_launch_us_steady": med(d[2:2 * K:2]), "head_us_steady": med(d[3:2 * K:2]),
            "flush_kernel_us": d[-1],
            "gap_fwd_to_head_us": med(gaps[0:2 * K - 1:2]),
            "gap_head_to_next_us": med(gaps[1:2 * K - 1:2]),
            "gap_before_flush_us": gaps[-1],
            "steps_1_2_us": (inside[4][0] - inside[0][0]) / 1e3,
            "steady_step_us": med([(inside[i + 2][0] - inside[i][0]) / 1e3
                                   for i in range(4, 2 * K - 2, 2)]),
        })
    out = {"K": K, "regions_matched": len(rows), "of": len(h["regions"])}
    if rows:
        out.update({k: med([r[k] for r in rows]) for k in rows[0]})
    print(json.dumps(out, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--analyze", nargs=2, metavar=("TRACE_CSV", "HOST_JSON"))
    ap.add_argument("--out", default="k20_host.json")
    ap.add_argument("--K", type=int, default=20)
    ap.add_argument("--reps", type=int, default=15)
    a = ap.parse_args()
    if a.analyze:
        analyze(*a.analyze)
    else:
        run(a.out, a.K, a.reps)


if __name__ == "__main__":
    main()
