#!/bin/bash
# PMC counters of the kernels matching KFILTER in one command (each counter pass its own run,
# killed if it hangs).  KFILTER=attn_bwd PMC_CMD="tools/probes/attn_one.py 20" scripts/gpu_pmc_kernel.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); OUT=$R/gpurun_out/pmc_${KFILTER:-all}; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o run -- python $R/$PMC_CMD > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  f=$(find "$OUT/p$i" -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && python - "$f" "${KFILTER:-}" <<'PY'
import csv, sys, collections, re
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(float); n = collections.Counter()
for r in rows:
    if sys.argv[2] not in r.get("Kernel_Name", ""): continue
    kn = re.sub(r"\(.*$", "", r["Kernel_Name"]).replace("void ", "").replace("dtfx::", "")[:60]
    key = (kn, r["Counter_Name"])
    agg[key] += float(r["Counter_Value"]); n[key] += 1
for k in sorted(agg): print("%-60s %-26s %16.0f  (%d dispatch rows)" % (k[0], k[1], agg[k], n[k]))
PY
done
