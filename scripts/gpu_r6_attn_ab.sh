#!/bin/bash
# Round 6: swizzled attention images (this tree) vs the padded 144-B rows (abtest/oldattn), same
# box: standalone attn_one interleaved, LDS-conflict PMC of both, BERT-base interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); OUT=$R/gpurun_out/r6attn; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_bert_gpu.py tests/test_bf16_gpu.py tests/test_transformer_gpu.py tests/test_kernels_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do for t in new old; do
  d=.; [ $t = old ] && d=abtest/oldattn
  timeout -k 10 120 python $d/tools/probes/attn_one.py 40 > $OUT/attn_${t}_$r.json 2>&1 || exit 1
  echo "$t $(tail -1 $OUT/attn_${t}_$r.json)"
done; done
for t in new old; do
  d=$R; [ $t = old ] && d=$R/abtest/oldattn
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/pmc_$t -o run -- python $d/tools/probes/attn_one.py 10 > $OUT/pmc_$t.log 2>&1) || { tail -5 $OUT/pmc_$t.log; exit 1; }
  f=$(find $OUT/pmc_$t -name "*counter_collection.csv" | head -1)
  python - "$f" > $OUT/pmc_$t.txt <<'PY'
import csv, sys, collections, re
agg = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "attn" not in r.get("Kernel_Name", ""): continue
    kn = re.sub(r"\(.*$", "", r["Kernel_Name"]).replace("void ", "").replace("dtfx::", "")[:40]
    agg[(kn, r["Counter_Name"])] += float(r["Counter_Value"])
for k in sorted(agg): print("%-40s %-26s %16.0f" % (k[0], k[1], agg[k]))
PY
  echo "== $t"; cat $OUT/pmc_$t.txt
done
for r in 1 2; do for t in new old; do
  d=.; [ $t = old ] && d=abtest/oldattn
  timeout -k 10 200 python $d/bench.py --model bert > $OUT/bert_${t}_$r.json 2>&1 || exit 1
  echo "bert $t $(tail -1 $OUT/bert_${t}_$r.json | cut -c 100-140)"
done; done
# MLP flush launch: the steps' own kernel instantiation vs the apply-only one
for r in 1 2; do for F in 1 0; do
  DTFX_MLP_FLUSH_FWD=$F timeout -k 10 200 python tools/probes/k20_split.py --reps 31 > $OUT/k20_flushfwd${F}_$r.json 2>&1 || exit 1
  echo "k20 flushfwd=$F $(tail -1 $OUT/k20_flushfwd${F}_$r.json | cut -c 1-200)"
done; done
for r in 1 2; do for F in 1 0; do
  DTFX_MLP_FLUSH_FWD=$F timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $OUT/bench_flushfwd${F}_$r.json 2>&1 || exit 1
  echo "bench flushfwd=$F $(tail -1 $OUT/bench_flushfwd${F}_$r.json | cut -c 1-110)"
done; done
# weight-gradient tiles (128x128 split-K / 256x128 / 8-phase) and the QKV auto choice
DTFX_GEMM_TA8=1 timeout -k 10 300 python tools/gemm_cfg_ab.py --cfgs 0,1,2,5 --rounds 5 --shapes ffn1_wgrad,qkv_wgrad,qkv_fwd > $OUT/gemm_wgrad.jsonl 2>&1 || exit 1
cut -c 1-220 $OUT/gemm_wgrad.jsonl
