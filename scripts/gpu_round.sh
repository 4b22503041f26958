#!/bin/bash
# One gpurun session: GPU tests, 1-GPU bench, rocprofv3 kernel stats.
# Stops at the first fault/abort/timeout (exit 124/134/137/139) -- never retries.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }

STEPS=${STEPS:-20000}
WARM=${WARM:-2000}
PROF_STEPS=${PROF_STEPS:-2000}

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests ${TEST_ARGS:--m gpu} -x -q -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu.log"
  if fatal $rc; then echo "FATAL in tests"; exit $rc; fi
fi

timeout -k 10 300 python bench.py --steps $STEPS --warmup $WARM ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.log" | tail -3
if [ $rc -ne 0 ]; then exit $rc; fi

if [ "${SKIP_PROF:-0}" != "1" ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
      python "$R/bench.py" --steps $PROF_STEPS --warmup 200 ${BENCH_ARGS:-} > "$OUT/prof.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 "$OUT/prof.log"
  find "$OUT/prof" -name "*stats*" | head
fi
