#!/bin/bash
# MI355X-native sync data parallelism: one process per GPU, RCCL/xGMI all-reduce.
nproc=${NPROC:-8}
cd "$(dirname "$0")"
exec python -m distributedtensorflowexample_amd.launch mirrored --nproc $nproc -- "$@"
