#!/bin/bash
# Hardware counters per kernel of the 1-GPU BERT-base step: three rocprofv3 --pmc passes (each
# its own run, killed if it hangs), joined by tools/pmc_summary.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); OUT=$R/gpurun_out/bert_pmc; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o run -- python "$R/tools/probes/dp_sim.py" --model bert --variants 1gpu --steps 3 --rounds 1 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
cd "$R"
python tools/pmc_summary.py "BERT-base step (seq 128, batch 128), 1 GPU" $(find "$OUT/p1" "$OUT/p2" "$OUT/p3" -name "*counter_collection.csv") > "$OUT/bert_pmc.md"
rm -f $(find "$OUT" -name "*counter_collection.csv")
head -30 "$OUT/bert_pmc.md"
