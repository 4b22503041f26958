set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_xgmi_gpu.py -k "factor or fused" -p no:cacheprovider > gpurun_out/t_factor.log 2>&1 || { echo FAIL tests; tail -30 gpurun_out/t_factor.log; exit 1; }
tail -8 gpurun_out/t_factor.log
DTFX_SHARED_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2000 --warmup 200 > gpurun_out/shared2.log 2>&1 || { echo FAIL shared; tail -30 gpurun_out/shared2.log; exit 1; }
tail -12 gpurun_out/shared2.log
