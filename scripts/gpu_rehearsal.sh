#!/bin/bash
# Multi-rank bench paths rehearsed on ONE GPU (ranks share device 0; an xGMI LL communicator
# stands in for RCCL).  Timings are not multi-GPU numbers; correctness + selection flow are.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/rehearsal; mkdir -p "$OUT"
for n in ${RANKS:-2 3}; do
  DTFX_WATCHDOG_S=${WATCHDOG:-150} DTFX_SHARED_GPU=1 timeout -k 10 ${TMO:-200} python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n \
    --steps ${STEPS:-2000} --warmup 200 ${BENCH_ARGS:-} > "$OUT/shared_mlp_$n.log" 2>&1
  rc=$?; echo "ranks=$n rc=$rc"; grep -E "probe|metric" "$OUT/shared_mlp_$n.log" | cut -c1-330
  [ $rc -ne 0 ] && { grep -v "amdgpu.ids\|hostname" "$OUT/shared_mlp_$n.log" | tail -30; exit $rc; }
done
exit 0
