#!/bin/bash
# Round 6: ResNet-50 -- the BatchNorm coefficients formed inside the 1x1 prologue kernels
# (DTFX_BN_COEF_FUSED) A/B'd end to end with a kernel-launch count, and the
# owner-sharded momentum SGD (DTFX_RESNET_ZERO1) in the simulated world-8 data-parallel shape
# (tools/probes/dp_sim.py); the ResNet / CNN GPU tests first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; OUT=gpurun_out/r6rz; mkdir -p $OUT
R=$PWD
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_cnn_gpu.py tests/test_resnet_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for r in 1 2 3; do for v in 1 0; do
  DTFX_BN_COEF_FUSED=$v timeout -k 10 300 python bench.py --model resnet50 > $OUT/resnet_f${v}_$r.json 2>&1 || { tail -5 $OUT/resnet_f${v}_$r.json; exit 1; }
  echo "resnet coef_fused=$v $r $(tail -1 $OUT/resnet_f${v}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/rprof" -o run -- python "$R/bench.py" --model resnet50 --steps 6 --warmup 3 > "$R/$OUT/rprof.log" 2>&1 || { tail -20 "$R/$OUT/rprof.log"; exit 1; }
cd "$R"
python tools/prof_summary.py $OUT/rprof/run_kernel_stats.csv 9 > $OUT/resnet_kernel_stats.txt && tail -1 $OUT/resnet_kernel_stats.txt
timeout -k 10 600 python tools/probes/dp_sim.py --model resnet50 --variants 1gpu,dp,dp_zero1,dp_null \
  --steps 10 --rounds 3 > $OUT/dp_sim_resnet.json 2> $OUT/dp_sim_resnet.err || { tail -20 $OUT/dp_sim_resnet.err; exit 1; }
cat $OUT/dp_sim_resnet.json
