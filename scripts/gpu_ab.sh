#!/bin/bash
# Interleaved A/B of environment knobs on one model's bench.py in one gpurun session (same box).
#   scripts/gpu_ab.sh MODEL ROUNDS "ENV_A=1" "ENV_A=0" ...
# prints "<knobs> <images|sequences|samples>/sec" per run; each run under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
model=$1; rounds=$2; shift 2
mkdir -p gpurun_out
for r in $(seq 1 "$rounds"); do
  for cfg in "$@"; do
    env $cfg timeout -k 10 200 python bench.py --model "$model" --steps 20 --warmup 5 \
      > gpurun_out/ab.log 2>&1 || exit 1
    v=$(tail -1 gpurun_out/ab.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')
    echo "round $r | $cfg | $v"
  done
done
