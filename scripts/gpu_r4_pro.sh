set -o pipefail
mkdir -p gpurun_out/pro
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cnn_gpu.py -k "prologue or stem or conv_fwd_dgrad_wgrad or fused_batchnorm" > gpurun_out/pro/t1.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_resnet_gpu.py tests/test_cnn_gpu.py > gpurun_out/pro/t2.log 2>&1 && \
timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/pro/bench_on.json 2> gpurun_out/pro/bench_on.err && \
DTFX_BN_PROLOGUE=0 DTFX_STEM_POOL_BN=0 timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/pro/bench_off.json 2> gpurun_out/pro/bench_off.err && \
timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/pro/bench_on2.json 2> gpurun_out/pro/bench_on2.err
echo rc=$?
