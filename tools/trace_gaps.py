"""Idle gaps and overlap in a rocprofv3 kernel_trace.csv: over the window between the
first and the last kernel whose name matches --window (e.g. the optimizer kernel that ends
every training step), print the span, the union of busy intervals, the idle time split
into gap-size buckets, the summed kernel time (> union when streams overlap) and the
largest gaps with the kernels on either side.

    python tools/trace_gaps.py gpurun_out/rprof/run_kernel_trace.csv --window sgd_momentum
"""
import argparse
import csv
import re


def short(name):
    name = re.sub(r"\(.*\)$", "", name).replace("void ", "").replace("dtfx::", "")
    return name[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window", default=None, help="kernel-name substring that ends a step")
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    ks = []
    for r in csv.DictReader(open(a.trace)):
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                   r.get("Queue_Id", r.get("Stream_Id", "?"))))
    ks.sort()
    if a.window:
        ends = [i for i, k in enumerate(ks) if a.window in k[2]]
        if len(ends) >= 2:
            ks = ks[ends[0] + 1:ends[-1] + 1]
            print("window: %d steps, %d kernels" % (len(ends) - 1, len(ks)))
    t0, t1 = ks[0][0], max(k[1] for k in ks)
    busy, cur_s, cur_e = 0, ks[0][0], ks[0][1]
    gaps = []
    prev = ks[0]
    for k in ks[1:]:
        if k[0] > cur_e:
            busy += cur_e - cur_s
            gaps.append((k[0] - cur_e, prev[2], k[2]))
            cur_s, cur_e = k[0], k[1]
        else:
            cur_e = max(cur_e, k[1])
        if k[1] >= cur_e:
            prev = k
    busy += cur_e - cur_s
    ksum = sum(k[1] - k[0] for k in ks)
    span = t1 - t0
    print("span %.3f ms  busy(union) %.3f ms (%.1f %%)  idle %.3f ms  sum of kernel times %.3f ms"
          % (span / 1e6, busy / 1e6, 100.0 * busy / span, (span - busy) / 1e6, ksum / 1e6))
    buckets = [(0, 2e3), (2e3, 5e3), (5e3, 10e3), (10e3, 50e3), (50e3, 1e12)]
    for lo, hi in buckets:
        g = [x[0] for x in gaps if lo <= x[0] < hi]
        print("  gaps %6.0f-%-8s us: %6d  total %.3f ms" % (lo / 1e3, "%.0f" % (hi / 1e3) if hi < 1e12 else "inf",
                                                          len(g), sum(g) / 1e6))
    print("largest gaps:")
    for g, p, n in sorted(gaps, reverse=True)[:a.top]:
        print("  %8.1f us  after %s  before %s" % (g / 1e3, short(p), short(n)))


if __name__ == "__main__":
    main()
