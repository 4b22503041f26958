"""Group a rocprofv3 kernel_trace.csv by (kernel, grid, workgroup) and print the time per
group: which GEMM shape / which launch configuration costs what, per dispatch.

    python tools/trace_by_shape.py gpurun_out/bprof/run_kernel_trace.csv [top]
"""
import collections
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(.*\)$", "", name)          # drop the parameter list
    name = name.replace("void ", "").replace("dtfx::", "")
    return name[:90]


def main(path, top=40):
    groups = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        key = (short(r["Kernel_Name"]), int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]),
               int(r["Grid_Size_Z"]), int(r["Workgroup_Size_X"]))
        groups[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tot = sum(sum(v) for v in groups.values())
    rows = sorted(groups.items(), key=lambda kv: -sum(kv[1]))[:top]
    print("%6s %10s %6s %9s %9s  %s" % ("%", "total_us", "calls", "avg_us", "min_us",
                                         "kernel [grid x,y,z / wg]"))
    for (name, gx, gy, gz, wg), v in rows:
        print("%6.2f %10.1f %6d %9.1f %9.1f  %s [%d,%d,%d / %d]" % (
            100 * sum(v) / tot, sum(v), len(v), sum(v) / len(v), min(v), name, gx, gy, gz, wg))
    print("total %.3f ms" % (tot / 1e3))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40)
