#!/bin/bash
# Interleaved end-to-end A/B of this tree against a modified copy built in abtest/<name>
# (same box, same inputs): bash scripts/gpu_tree_ab.sh <name> "<bench args>" [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NAME=$1; ARGS=$2; ROUNDS=${3:-3}
OUT=gpurun_out/tree_ab/$NAME; mkdir -p $OUT
tag=$(echo "$ARGS" | tr -c 'a-z0-9' '_')
for r in $(seq 1 $ROUNDS); do
  for t in base $NAME; do
    script=bench.py; [ $t != base ] && script=abtest/$NAME/bench.py
    timeout -k 10 200 python $script $ARGS > $OUT/${t}_${tag}_$r.json 2>/dev/null || exit 1
    echo "[$t $ARGS] round=$r $(tail -1 $OUT/${t}_${tag}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
