#!/bin/bash
# Reference run_multi_gpu.sh: 1 ps + 16 workers on 4 GPUs (4 per GPU, async PS).
num_workers=16
num_gpus=4
GPU_ID=(0 1 2 3)
cd "$(dirname "$0")"
exec python -m distributedtensorflowexample_amd.launch ps --num_workers $num_workers \
    --num_gpus $num_gpus --gpu_ids "$(IFS=,; echo "${GPU_ID[*]}")" -- "$@"
