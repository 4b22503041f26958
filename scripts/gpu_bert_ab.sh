set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u -m pytest -x -q --timeout 60 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py -k host_loop > gpurun_out/t_hl.log 2>&1; tail -1 gpurun_out/t_hl.log
for big in 5 3; do for ws in 1 0; do
  DTFX_GEMM_BIG=$big DTFX_BERT_WSTREAM=$ws timeout -k 10 200 python bench.py --model bert > gpurun_out/bb.log 2>&1 || exit 1
  echo "big=$big wstream=$ws $(tail -1 gpurun_out/bb.log | cut -c 80-150)"
done; done
cd /tmp && DTFX_BERT_WSTREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/bprof5 -o run -- python $GRAFT_REPO_ROOT/bench.py --model bert --steps 6 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/bprof5.log 2>&1 || exit 1
python $GRAFT_REPO_ROOT/tools/trace_by_shape.py $GRAFT_REPO_ROOT/gpurun_out/bprof5/run_kernel_trace.csv 25 > $GRAFT_REPO_ROOT/gpurun_out/bprof5_shapes.txt
