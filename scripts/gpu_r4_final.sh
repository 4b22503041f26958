# Round-4 final check with the tree as committed: smoke + the whole GPU tier (as the driver runs them)
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/final/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python bench.py > gpurun_out/final/bench_mlp_default.json 2>&1 || exit 1
echo done
