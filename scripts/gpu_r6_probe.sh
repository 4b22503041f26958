#!/bin/bash
# Round-6 probe: K=20 region split (completion waits), MLP benches, ZeRO-1 BERT DP shape.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; OUT=gpurun_out/r6probe2; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_xgmi_sim_gpu.py -k "bw" tests/test_bert_gpu.py tests/test_bf16_gpu.py tests/test_transformer_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 120 python tools/probes/attn_one.py 40 > $OUT/attn_one.json 2>&1 || { tail $OUT/attn_one.json; exit 1; }
tail -1 $OUT/attn_one.json
timeout -k 10 200 python tools/probes/k20_split.py > $OUT/k20_split.json 2>&1 || { tail $OUT/k20_split.json; exit 1; }
tail -1 $OUT/k20_split.json
for i in 1 2 3; do timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $OUT/k20_$i.json 2>&1 || exit 1; tail -1 $OUT/k20_$i.json | cut -c 1-100; done
for T in 1 0; do DTFX_GEMM_TAILSPLIT=$T timeout -k 10 300 python tools/gemm_cfg_ab.py --cfgs 5 --rounds 5 --shapes qkv_fwd > $OUT/gemm_qkv_tail$T.jsonl 2>&1 || exit 1; cut -c 1-160 $OUT/gemm_qkv_tail$T.jsonl | tail -1; done
for i in 1 2; do for T in 1 0; do DTFX_GEMM_TAILSPLIT=$T timeout -k 10 200 python bench.py --model bert > $OUT/bert_tail${T}_$i.json 2>&1 || exit 1; echo tail=$T; tail -1 $OUT/bert_tail${T}_$i.json | cut -c 1-110; done; done
timeout -k 10 600 python -u tools/probes/dp_sim.py --model bert --world 8 --steps 10 --rounds 2 --variants 1gpu,dp,dp_rep > $OUT/dp_sim_bert.jsonl 2>&1 || { tail -20 $OUT/dp_sim_bert.jsonl; exit 1; }
tail -5 $OUT/dp_sim_bert.jsonl
