"""Kernel-by-kernel difference of two rocprofv3 --stats runs (kernel_stats.csv), per step:

    python tools/kernel_stats_diff.py A.csv STEPS_A B.csv STEPS_B [top]

STEPS may be a number or ``k=<substring>``: the call count of the (first) kernel whose name
contains the substring -- one that runs exactly once per step, so warm-up and capture steps
are counted the same way in both runs.

Prints us/step of every kernel in A and B and B - A, sorted by |B - A|, then the totals --
e.g. the 1-GPU BERT step against its simulated world-8 data-parallel shape
(tools/probes/dp_sim.py): which kernels the DP mode adds (the all-reduce) and which of the
step's own kernels it slows down (contention with them)."""
import csv
import sys


def load(path, steps):
    out = {}
    rows = list(csv.DictReader(open(path)))
    if steps.startswith("k="):
        steps = next(float(r["Calls"]) for r in rows if steps[2:] in r["Name"])
        print("%s: %d steps" % (path, steps))
    steps = float(steps)
    for r in rows:
        out[r["Name"]] = out.get(r["Name"], 0.0) + float(r["TotalDurationNs"]) / 1e3 / steps
    return out


def main():
    a, sa, b, sb = sys.argv[1:5]
    top = int(sys.argv[5]) if len(sys.argv) > 5 else 25
    A, B = load(a, sa), load(b, sb)
    names = sorted(set(A) | set(B), key=lambda n: -abs(B.get(n, 0.0) - A.get(n, 0.0)))
    print("%10s %10s %10s  kernel" % ("A us/step", "B us/step", "B - A"))
    for n in names[:top]:
        x, y = A.get(n, 0.0), B.get(n, 0.0)
        print("%10.1f %10.1f %+10.1f  %s" % (x, y, y - x, n[:110]))
    ta, tb = sum(A.values()), sum(B.values())
    print("%10.1f %10.1f %+10.1f  TOTAL kernel time per step" % (ta, tb, tb - ta))


if __name__ == "__main__":
    main()
