#!/bin/bash
# Round 6: ResNet-50 owner-sharded momentum SGD (DTFX_RESNET_ZERO1) in the simulated world-8
# data-parallel shape (tools/probes/dp_sim.py), the ResNet GPU tests, the 1-GPU bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; OUT=gpurun_out/r6rz; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_resnet_gpu.py tests/test_cnn_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 600 python tools/probes/dp_sim.py --model resnet50 --variants 1gpu,dp,dp_zero1,dp_null \
  --steps 10 --rounds 3 > $OUT/dp_sim_resnet.json 2> $OUT/dp_sim_resnet.err || { tail -20 $OUT/dp_sim_resnet.err; exit 1; }
cat $OUT/dp_sim_resnet.json
timeout -k 10 300 python bench.py --model resnet50 > $OUT/bench_resnet.json 2>&1 || { tail -5 $OUT/bench_resnet.json; exit 1; }
tail -1 $OUT/bench_resnet.json
