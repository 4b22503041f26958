#!/bin/bash
# Memory-path PMC counters (L2 / HBM requests) of the kernels matching KFILTER under PMC_CMD,
# each pass its own run, killed if it hangs.
#   KFILTER=conv1x1 PMC_CMD="tools/probes/conv_one.py fwd 256 56 56 64 256 1 1 0" scripts/gpu_pmc_mem.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); OUT=$R/gpurun_out/pmcm_${TAG:-${KFILTER:-all}}; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
i=0
for set in "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" \
           "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_WRITE_sum" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o run -- python $R/$PMC_CMD > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  f=$(find "$OUT/p$i" -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && python - "$f" "${KFILTER:-}" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(float); n = collections.Counter()
for r in rows:
    if sys.argv[2] not in r.get("Kernel_Name", ""): continue
    agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(agg): print("%-28s %16.0f  (%d dispatch rows)" % (k, agg[k], n[k]))
PY
done
