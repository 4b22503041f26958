"""Summarize a rocprofv3 --stats kernel_stats.csv (or the rocpd SQLite database rocprofv3
writes without --output-format csv): top kernels by total time."""
import csv
import sqlite3
import sys


def _rows(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        return [{"Name": n, "Calls": str(k), "TotalDurationNs": float(t) * 1e3,
                 "AverageNs": float(a) * 1e3}
                for n, k, t, a in c.execute(
                    "select name, total_calls, total_duration, average from top_kernels")]
    return list(csv.DictReader(open(path)))


def main(path, top=25, steps=None):
    rows = _rows(path)
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    out = []
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        out.append("%6.2f%% %11.1f us  calls=%6s  avg=%9.1f us  %s" % (
            100 * float(r["TotalDurationNs"]) / tot, float(r["TotalDurationNs"]) / 1e3, r["Calls"],
            float(r["AverageNs"]) / 1e3, r["Name"][:120]))
    out.append("total kernel time: %.3f ms%s" % (tot / 1e6, "" if not steps else
                                                 " (%.3f ms/step over %d steps)" % (tot / 1e6 / steps, steps)))
    return "\n".join(out)


if __name__ == "__main__":
    print(main(sys.argv[1], steps=int(sys.argv[2]) if len(sys.argv) > 2 else None))
