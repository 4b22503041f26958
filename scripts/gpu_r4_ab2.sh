# Round-4 A/B: BERT weight gradients issued per layer (one cross-stream edge) vs per GEMM;
# the stem weight gradient forming dL/dc in its staging vs the separate apply pass
set -o pipefail
mkdir -p gpurun_out/ab2
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cnn_gpu.py tests/test_resnet_gpu.py tests/test_bert_gpu.py > gpurun_out/ab2/t.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python bench.py --model bert > gpurun_out/ab2/bert_batch_$r.json 2>/dev/null || exit 1
  DTFX_BERT_WGRAD_BATCH=0 timeout -k 10 300 python bench.py --model bert > gpurun_out/ab2/bert_pergemm_$r.json 2>/dev/null || exit 1
done
for r in 1 2; do
  timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/ab2/resnet_on_$r.json 2>/dev/null || exit 1
  DTFX_STEM_WGRAD_BN=0 timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/ab2/resnet_off_$r.json 2>/dev/null || exit 1
done
echo done
