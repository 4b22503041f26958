"""Kernel-by-kernel difference of two rocprofv3 --stats runs (kernel_stats.csv), per step:

    python tools/kernel_stats_diff.py A.csv STEPS_A B.csv STEPS_B [top]

Prints us/step of every kernel in A and B and B - A, sorted by |B - A|, then the totals --
e.g. the 1-GPU BERT step against its simulated world-8 data-parallel shape
(tools/probes/dp_sim.py): which kernels the DP mode adds (the all-reduce) and which of the
step's own kernels it slows down (contention with them)."""
import csv
import sys


def load(path, steps):
    out = {}
    for r in csv.DictReader(open(path)):
        out[r["Name"]] = out.get(r["Name"], 0.0) + float(r["TotalDurationNs"]) / 1e3 / steps
    return out


def main():
    a, sa, b, sb = sys.argv[1], float(sys.argv[2]), sys.argv[3], float(sys.argv[4])
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
