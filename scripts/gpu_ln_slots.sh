set -o pipefail
mkdir -p gpurun_out/ln
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -k layernorm -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ln/pytest.log 2>&1 || { tail -30 gpurun_out/ln/pytest.log; exit 1; }
tail -1 gpurun_out/ln/pytest.log
timeout -k 10 120 python tools/probes/ln_bwd_slots.py > gpurun_out/ln/ln_bwd_slots.json 2>&1 || { tail -20 gpurun_out/ln/ln_bwd_slots.json; exit 1; }
tail -1 gpurun_out/ln/ln_bwd_slots.json
for r in 1 2 3; do
  for s in 2 3; do
    DTFX_LN_SLOTS=$s timeout -k 10 200 python bench.py --model bert > gpurun_out/ln/bert_s${s}_$r.json 2>&1 || exit 1
    echo "round $r slots $s $(tail -1 gpurun_out/ln/bert_s${s}_$r.json | cut -c 1-140)"
  done
done
