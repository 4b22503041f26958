"""Per-kernel hardware-counter summary from several rocprofv3 ``--pmc`` passes of the same
deterministic workload (scripts/gpu_pmc.sh: one pass per counter group, each its own run).

    python tools/pmc_summary.py <title> <pass1/..._counter_collection.csv> [<pass2> ...]

Dispatches are grouped by (kernel, grid, workgroup); counters are averaged per dispatch in
each pass and the passes joined on that key.  Derived columns:

* ``mfma%``  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs)
              (rocprof's MfmaUtil; GRBM_GUI_ACTIVE is reported summed over the 8 XCDs)
* ``lds_cf%`` = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles per LDS cycle)
* ``rd GB/s`` = 2 * FETCH_SIZE KB / duration (gfx950 FETCH_SIZE counts half of the bytes of
              wide coalesced reads -- MI355X_MICROARCH.md; an upper estimate for narrow ones)
* ``wr GB/s`` = WRITE_SIZE KB / duration;  ``L2 hit%`` = TCC_HIT / (TCC_HIT + TCC_MISS)
* ``clk GHz`` = GRBM_GUI_ACTIVE / 8 / duration (reads high below ~0.3 ms dispatches)
Durations are the PMC runs' own dispatch timestamps (profiled runs clock lower than
un-profiled ones).
"""
import collections
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(.*\)$", "", name).replace("void ", "").replace("dtfx::", "")
    return name[:70]


def load(path):
    """{key: {counter: mean per dispatch, '_dur_ns': mean, '_n': dispatches}}"""
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        key = (short(r["Kernel_Name"]), int(r["Grid_Size"]), int(r["Workgroup_Size"]))
        did = r["Dispatch_Id"]
        per[key][r["Counter_Name"]].append((did, float(r["Counter_Value"])))
        durs[key][did] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = {}
    for key, cs in per.items():
        d = {}
        for c, vals in cs.items():
            byd = collections.defaultdict(float)
            for did, v in vals:  # several rows per dispatch (per XCD / instance) are summed
                byd[did] += v
            d[c] = sum(byd.values()) / len(byd)
        d["_n"] = len(durs[key])
        d["_dur_ns"] = sum(durs[key].values()) / len(durs[key])
        out[key] = d
    return out


def main(title, paths):
    merged = collections.defaultdict(dict)
    for p in paths:
        for key, d in load(p).items():
            m = merged[key]
            for c, v in d.items():
                if c == "_dur_ns":
                    m.setdefault("_durs", []).append(v)
                else:
                    m[c] = v
    rows = []
    for key, m in merged.items():
        dur = sum(m["_durs"]) / len(m["_durs"])  # ns
        g = m.get("GRBM_GUI_ACTIVE")
        cyc = g / 8.0 if g else None
        def pct(a, b):
            return 100.0 * a / b if (a is not None and b) else None
        rows.append((dur * m.get("_n", 1), key, {
            "n": m.get("_n"), "us": dur / 1e3,
            "mfma%": pct(m.get("SQ_VALU_MFMA_BUSY_CYCLES"), cyc * 1024 if cyc else None),
            "mfma_inst": m.get("SQ_INSTS_MFMA"),
            "lds_cf%": pct(m.get("SQ_LDS_BANK_CONFLICT"), m.get("SQ_LDS_IDX_ACTIVE")),
            "rd GB/s": (2 * m["FETCH_SIZE"] * 1024 / dur) if "FETCH_SIZE" in m else None,
            "wr GB/s": (m["WRITE_SIZE"] * 1024 / dur) if "WRITE_SIZE" in m else None,
            "L2 hit%": pct(m.get("TCC_HIT_sum"),
                           (m.get("TCC_HIT_sum") or 0) + (m.get("TCC_MISS_sum") or 0)),
            "clk GHz": (cyc / dur) if cyc else None,
        }))
    rows.sort(key=lambda r: -r[0])
    cols = ["n", "us", "mfma%", "mfma_inst", "lds_cf%", "rd GB/s", "wr GB/s", "L2 hit%", "clk GHz"]
    print("### %s\n" % title)
    print("| kernel [grid / wg] | " + " | ".join(cols) + " |")
    print("|---" * (len(cols) + 1) + "|")
    for _, (name, grid, wg), v in rows[:25]:
        cells = []
        for c in cols:
            x = v[c]
            cells.append("-" if x is None else ("%d" % x if c in ("n", "mfma_inst") else
                                                "%.1f" % x if c != "clk GHz" else "%.2f" % x))
        print("| `%s` [%d / %d] | %s |" % (name, grid, wg, " | ".join(cells)))
    print()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
