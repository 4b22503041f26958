#!/bin/bash
# Reference run_single_gpu.sh: 1 ps + 2 workers sharing GPU 0 (async PS SGD).
# tmux windows are replaced by the Python launcher (one log per task under
# launch_logs/, streamed with [task] prefixes).  Extra main.py flags after --.
num_workers=2
num_gpus=1
GPU_ID=(0)
cd "$(dirname "$0")"
exec python -m distributedtensorflowexample_amd.launch ps --num_workers $num_workers \
    --num_gpus $num_gpus --gpu_ids "$(IFS=,; echo "${GPU_ID[*]}")" -- "$@"
