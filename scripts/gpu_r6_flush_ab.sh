#!/bin/bash
# Round 6: the driver-sized MLP region with the flush folded into the last step's head
# (mlp_head_flush_kernel, DTFX_MLP_FLUSH_FUSED=1, default) against the separate flush launch
# (=0), interleaved on one box; host-side settings beside them; then the BERT step's kernel
# stats (hand-written GEMMs only: no Cijk_ kernel may appear).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; OUT=gpurun_out/r6flush; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "terminal_head_flush or host_loop_matches" > $OUT/pytest.log 2>&1 \
  || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for r in 1 2 3 4 5 6; do
  for v in fused sep devkarg0 spin; do
    case $v in
      fused) E="DTFX_MLP_FLUSH_FUSED=1" ;; sep) E="DTFX_MLP_FLUSH_FUSED=0" ;;
      devkarg0) E="HIP_FORCE_DEV_KERNARG=0" ;; spin) E="DTFX_HIP_SCHED=spin" ;;
    esac
    [ $r -gt 3 ] && [ $v != fused ] && [ $v != sep ] && continue
    env $E timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $OUT/${v}_$r.json 2>&1 || { tail -5 $OUT/${v}_$r.json; exit 1; }
    echo "$v $r $(tail -1 $OUT/${v}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
if [ "${BERT_PROF:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bert_prof -o bert -- \
    python bench.py --model bert --steps 8 --warmup 3 > $OUT/bert_prof.log 2>&1 || { tail -20 $OUT/bert_prof.log; exit 1; }
  tail -1 $OUT/bert_prof.log
fi
