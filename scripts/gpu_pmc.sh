#!/bin/bash
# Hardware counters (rocprofv3 --pmc, no tracing) of the framework's hot kernels:
# peak bf16 GEMM, BERT FFN GEMM, MNIST-MLP step, BERT-base and ResNet-50 training steps.
# Three passes per workload, each its own run under a hard time limit (counter slots per
# pass: 8 SQ + 1 GRBM | FETCH_SIZE (3 TCC) + 1 GRBM | WRITE_SIZE (2 TCC) + TCC_HIT/MISS).
# Summaries: gpurun_out/pmc2/summary.md (tools/pmc_summary.py).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); OUT=$R/gpurun_out/pmc2; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P2="FETCH_SIZE GRBM_GUI_ACTIVE"
P3="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
declare -A WL=(
  [gemm8192]="$R/tools/gemm_one.py 8192 8192 8192 0 1"
  [gemm_ffn1]="$R/tools/gemm_one.py 16384 3072 768 0 0"
  [mlp]="$R/bench.py --steps 300 --warmup 50 --no_graph"
  [bert]="$R/bench.py --model bert --steps 2 --warmup 1 --no_graph"
  [resnet50]="$R/bench.py --model resnet50 --steps 2 --warmup 1 --no_graph"
)
: > "$OUT/summary.md"
for w in ${WORKLOADS:-gemm8192 gemm_ffn1 mlp bert resnet50}; do
  files=()
  for i in 1 2 3; do
    eval "set=\$P$i"
    d="$OUT/$w/p$i"
    timeout -s KILL ${PASS_TIMEOUT:-150} rocprofv3 --pmc $set --output-format csv -d "$d" -o run -- \
      python3 ${WL[$w]} > "$OUT/$w.p$i.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$w pass $i failed rc=$rc"; tail -5 "$OUT/$w.p$i.log"; exit $rc; fi
    f=$(find "$d" -name "*counter_collection.csv" | head -1)
    [ -n "$f" ] && files+=("$f")
  done
  python3 "$R/tools/pmc_summary.py" "$w" "${files[@]}" >> "$OUT/summary.md" 2>&1
  echo "$w ok"
done
head -c 6000 "$OUT/summary.md"
