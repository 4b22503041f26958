#!/bin/bash
# Reference-equivalent async-PS baseline on the MI355X + kernel profile of the sync-DP bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python tools/bench_ps_async.py --num_workers 2 --steps 20000 --log_every 2000 > "$OUT/ps_async_w2.json" 2> "$OUT/ps_async_w2.err" && cat "$OUT/ps_async_w2.json" &&
timeout -k 10 600 python tools/bench_ps_async.py --num_workers 8 --steps 20000 --log_every 2000 --base_port 25222 > "$OUT/ps_async_w8.json" 2> "$OUT/ps_async_w8.err" && cat "$OUT/ps_async_w8.json" &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_dp1" -o run -- python "$OLDPWD/bench.py" --steps 5000 --warmup 500 > "$OUT/prof_dp1.log" 2>&1 && tail -1 "$OUT/prof_dp1.log" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_dpmode" -o run -- python "$OLDPWD/bench.py" --dp --steps 5000 --warmup 500 > "$OUT/prof_dpmode.log" 2>&1 && tail -1 "$OUT/prof_dpmode.log"
