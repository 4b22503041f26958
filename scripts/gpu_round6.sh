#!/bin/bash
# Round-6 GPU experiments in one parametrized driver (each was a one-off script):
#   bash scripts/gpu_round6.sh <experiment>
# Every experiment writes under gpurun_out/ and stops at its first failure.  Their results
# are in profiles/r6/ (each README names the experiment that produced it).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD

exp_flush() {
# Round 6: the driver-sized MLP region with the flush folded into the last step's head
# (mlp_head_flush_kernel, DTFX_MLP_FLUSH_FUSED=1, default) against the separate flush launch
# (=0), interleaved on one box; host-side settings beside them; then the BERT step's kernel
# stats (hand-written GEMMs only: no Cijk_ kernel may appear).
cd "$ROOT"; OUT=gpurun_out/r6flush; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "terminal_head_flush or host_loop_matches" > $OUT/pytest.log 2>&1 \
  || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for r in 1 2 3 4 5 6; do
  for v in fused sep devkarg0 spin; do
    case $v in
      fused) E="DTFX_MLP_FLUSH_FUSED=1" ;; sep) E="DTFX_MLP_FLUSH_FUSED=0" ;;
      devkarg0) E="HIP_FORCE_DEV_KERNARG=0" ;; spin) E="DTFX_HIP_SCHED=spin" ;;
    esac
    [ $r -gt 3 ] && [ $v != fused ] && [ $v != sep ] && continue
    env $E timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $OUT/${v}_$r.json 2>&1 || { tail -5 $OUT/${v}_$r.json; exit 1; }
    echo "$v $r $(tail -1 $OUT/${v}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
if [ "${BERT_PROF:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bert_prof -o bert -- \
    python bench.py --model bert --steps 8 --warmup 3 > $OUT/bert_prof.log 2>&1 || { tail -20 $OUT/bert_prof.log; exit 1; }
  tail -1 $OUT/bert_prof.log
fi
}

exp_pers() {
# Round 6: the persistent 8-phase tile loop (DTFX_GEMM_PERS, gemm_bf16.hip) -- GEMM tests,
# per-call A/B on the BERT shapes, then BERT-base and ResNet-50 end to end, interleaved.
cd "$ROOT"; OUT=gpurun_out/r6pers; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_bf16_gpu.py tests/test_bert_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python tools/probes/gemm_pers_ab.py > $OUT/gemm_pers_ab.jsonl 2>&1 || { tail -20 $OUT/gemm_pers_ab.jsonl; exit 1; }
cat $OUT/gemm_pers_ab.jsonl
for r in 1 2 3; do for v in 1 0; do
  DTFX_GEMM_PERS=$v timeout -k 10 200 python bench.py --model bert > $OUT/bert_p${v}_$r.json 2>&1 || { tail -5 $OUT/bert_p${v}_$r.json; exit 1; }
  echo "bert pers=$v $r $(tail -1 $OUT/bert_p${v}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
}

exp_resnet_zero1() {
# Round 6: ResNet-50 -- the BatchNorm coefficients formed inside the 1x1 prologue kernels
# (DTFX_BN_COEF_FUSED) A/B'd end to end with a kernel-launch count, and the
# owner-sharded momentum SGD (DTFX_RESNET_ZERO1) in the simulated world-8 data-parallel shape
# (tools/probes/dp_sim.py); the ResNet / CNN GPU tests first.
cd "$ROOT"; OUT=gpurun_out/r6rz; mkdir -p $OUT
R=$PWD
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_cnn_gpu.py tests/test_resnet_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for r in 1 2 3; do for v in 1 0; do
  DTFX_BN_COEF_FUSED=$v timeout -k 10 300 python bench.py --model resnet50 > $OUT/resnet_f${v}_$r.json 2>&1 || { tail -5 $OUT/resnet_f${v}_$r.json; exit 1; }
  echo "resnet coef_fused=$v $r $(tail -1 $OUT/resnet_f${v}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/rprof" -o run -- python "$R/bench.py" --model resnet50 --steps 6 --warmup 3 > "$R/$OUT/rprof.log" 2>&1 || { tail -20 "$R/$OUT/rprof.log"; exit 1; }
cd "$R"
python tools/prof_summary.py $OUT/rprof/run_kernel_stats.csv 9 > $OUT/resnet_kernel_stats.txt && tail -1 $OUT/resnet_kernel_stats.txt
timeout -k 10 600 python tools/probes/dp_sim.py --model resnet50 --variants 1gpu,dp,dp_zero1,dp_null \
  --steps 10 --rounds 3 > $OUT/dp_sim_resnet.json 2> $OUT/dp_sim_resnet.err || { tail -20 $OUT/dp_sim_resnet.err; exit 1; }
cat $OUT/dp_sim_resnet.json
}

exp_resnet_fold() {
# Round 6: ResNet-50 split-K weight gradients folded into momentum SGD (DTFX_RESNET_FOLD,
# VERDICT r5 item 7) -- tests, interleaved A/B, launch count; BERT weight gradients on the
# 8-phase tile (DTFX_GEMM_TA8) re-checked on this round's kernels.
cd "$ROOT"; OUT=gpurun_out/r6fold; mkdir -p $OUT
R=$PWD
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_resnet_gpu.py tests/test_cnn_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for r in 1 2 3; do for v in 1 0; do
  DTFX_RESNET_FOLD=$v timeout -k 10 300 python bench.py --model resnet50 > $OUT/resnet_fold${v}_$r.json 2>&1 || { tail -5 $OUT/resnet_fold${v}_$r.json; exit 1; }
  echo "resnet fold=$v $r $(tail -1 $OUT/resnet_fold${v}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/rprof" -o run -- python "$R/bench.py" --model resnet50 --steps 6 --warmup 3 > "$R/$OUT/rprof.log" 2>&1 || { tail -20 "$R/$OUT/rprof.log"; exit 1; }
cd "$R"
python tools/prof_summary.py $OUT/rprof/run_kernel_stats.csv 9 > $OUT/resnet_kernel_stats.txt && tail -1 $OUT/resnet_kernel_stats.txt
for r in 1 2; do for v in 0 1; do
  DTFX_GEMM_TA8=$v timeout -k 10 200 python bench.py --model bert > $OUT/bert_ta8_${v}_$r.json 2>&1 || { tail -5 $OUT/bert_ta8_${v}_$r.json; exit 1; }
  echo "bert ta8=$v $r $(tail -1 $OUT/bert_ta8_${v}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
}

exp_attn_rp() {
# Round 6: attention forward with P in registers (attn_fwd_rp_kernel, DTFX_ATTN_FWD) -- tests,
# per-call time against the P-through-LDS kernel, BERT-base end to end interleaved.
cd "$ROOT"; OUT=gpurun_out/r6attn; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_transformer_gpu.py tests/test_bert_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for r in 1 2 3; do for v in 1 0; do
  DTFX_ATTN_FWD=$v timeout -k 10 100 python tools/probes/attn_one.py 50 > $OUT/attn_one_f${v}_$r.json 2>&1 || { tail -5 $OUT/attn_one_f${v}_$r.json; exit 1; }
  echo "attn fwd=$v $r $(tail -1 $OUT/attn_one_f${v}_$r.json)"
done; done
for r in 1 2 3; do for v in 1 0; do
  DTFX_ATTN_FWD=$v timeout -k 10 200 python bench.py --model bert > $OUT/bert_f${v}_$r.json 2>&1 || { tail -5 $OUT/bert_f${v}_$r.json; exit 1; }
  echo "bert attn_fwd=$v $r $(tail -1 $OUT/bert_f${v}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
}

exp_k20_env() {
# Round 6: the driver-sized MLP bench under host-side settings, interleaved on one box.
cd "$ROOT"; OUT=gpurun_out/r6k20env; mkdir -p $OUT
for r in 1 2 3 4 5; do
  for v in base devkarg0 pin spin; do
    case $v in
      base) E="" ;; devkarg0) E="HIP_FORCE_DEV_KERNARG=0" ;; pin) E="DTFX_BENCH_PIN=1" ;; spin) E="DTFX_HIP_SCHED=spin" ;;
    esac
    env $E timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $OUT/${v}_$r.json 2>&1 || { tail -5 $OUT/${v}_$r.json; exit 1; }
    echo "$v $r $(tail -1 $OUT/${v}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["launch"])')"
  done
done
# BERT: weight gradients on the 8-phase tile (both operands transposed) vs 128x128 split-K
for r in 1 2; do for v in base ta8 ta8s128; do
  case $v in base) E="" ;; ta8) E="DTFX_GEMM_TA8=1" ;; ta8s128) E="DTFX_GEMM_TA8=1 DTFX_GEMM_TA8_SLOTS=128" ;; esac
  env $E timeout -k 10 200 python bench.py --model bert > $OUT/bert_${v}_$r.json 2>&1 || { tail -5 $OUT/bert_${v}_$r.json; exit 1; }
  echo "bert $v $r $(tail -1 $OUT/bert_${v}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
}

exp_probe() {
# Round-6 probe: K=20 region split (completion waits), MLP benches, ZeRO-1 BERT DP shape.
cd "$ROOT"; OUT=gpurun_out/r6probe2; mkdir -p $OUT; export TMPDIR=/tmp
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
}

exp_attn_swz() {
# Round 6: swizzled attention images (this tree) vs the padded 144-B rows (abtest/oldattn), same
# box: standalone attn_one interleaved, LDS-conflict PMC of both, BERT-base interleaved.
cd "$ROOT"; R=$(pwd); OUT=$R/gpurun_out/r6attn; mkdir -p $OUT; export TMPDIR=/tmp
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
}

exp_resnet_wt() {
# Round 6: the 1x1 data gradients' transposed weights formed by ONE batched launch per step
# (ResNet50._transpose_weights) instead of one transpose launch per dgrad -- tests, then
# ResNet-50 end to end against the previous tree state (DTFX_RESNET_WT_BATCH=0), interleaved.
cd "$ROOT"; OUT=gpurun_out/r6wt; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_resnet_gpu.py tests/test_cnn_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for r in 1 2 3; do for v in 1 0; do
  DTFX_RESNET_WT_BATCH=$v timeout -k 10 300 python bench.py --model resnet50 > $OUT/resnet_wt${v}_$r.json 2>&1 || { tail -5 $OUT/resnet_wt${v}_$r.json; exit 1; }
  echo "resnet wt_batch=$v $r $(tail -1 $OUT/resnet_wt${v}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
}

exp_mlp_plan() {
# Round 6: the MLP host loop's buffers bound once in a C++ plan (7-argument call before the
# region's first kernel instead of 17) -- host-loop tests, then the driver-sized bench
# interleaved against the 17-argument entry point (DTFX_MLP_PLAN=0).
cd "$ROOT"; OUT=gpurun_out/r6plan; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "host_loop or terminal_head_flush" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for r in 1 2 3 4 5 6; do for v in 1 0; do
  DTFX_MLP_PLAN=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $OUT/k20_plan${v}_$r.json 2>&1 || { tail -5 $OUT/k20_plan${v}_$r.json; exit 1; }
  echo "plan=$v $r $(tail -1 $OUT/k20_plan${v}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["launch"])')"
done; done
}

exp_zero_ranges() {
# Round 6: BERT's per-step gradient zeroing as ONE zero_ranges launch (DTFX_ZERO_RANGES) --
# BERT GPU tests, then BERT-base end to end interleaved.
cd "$ROOT"; OUT=gpurun_out/r6zero; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_bert_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for r in 1 2 3; do for v in 1 0; do
  DTFX_ZERO_RANGES=$v timeout -k 10 200 python bench.py --model bert > $OUT/bert_z${v}_$r.json 2>&1 || { tail -5 $OUT/bert_z${v}_$r.json; exit 1; }
  echo "bert zero_ranges=$v $r $(tail -1 $OUT/bert_z${v}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
}

exp_engines() {
# Round 6: the MLP exchange engines' local cost at world 2 / 4 / 8 (simulated peers,
# tools/probes/engine_local_cost.py) -- the xGMI simulation tests with the variant's
# DTFX_XG_SPLIT first, then the default (${BASE_SPLIT:-3}) and the variant (${VAR_SPLIT:-19})
# interleaved on one box.
cd "$ROOT"; OUT=gpurun_out/r6eng; mkdir -p $OUT
DTFX_XG_SPLIT=${VAR_SPLIT:-19} timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider tests/test_xgmi_sim_gpu.py > $OUT/xgmi_sim_${VAR_SPLIT:-19}.log 2>&1 || { tail -30 $OUT/xgmi_sim_${VAR_SPLIT:-19}.log; exit 1; }
tail -1 $OUT/xgmi_sim_${VAR_SPLIT:-19}.log
for r in 1 2 3; do for v in ${BASE_SPLIT:-3} ${VAR_SPLIT:-19}; do
  DTFX_XG_SPLIT=$v ENGINES=${ENGINES:-fused2x} timeout -k 10 200 python tools/probes/engine_local_cost.py > $OUT/elc_${v}_$r.json 2>$OUT/elc_${v}_$r.err || { tail -5 $OUT/elc_${v}_$r.err; exit 1; }
  echo "split=$v $r $(python -c "import json;d=json.load(open('$OUT/elc_${v}_$r.json'));print(d['single_gpu_2launch_us'],{e:[d['world%d'%w][e] for w in (2,4,8)] for e in d['world2'] if e!='epoch_reset_us'})")"
done; done
}

exp_attn_pf() {
# Round 6: the two-halves attention backward with the block's V rows requested at its start
# (L2 warm-up, DTFX_ATTN_BWD_PF=1, opt-in) against without (=0) -- attention GPU tests, the
# standalone probe and BERT-base end to end, interleaved.
cd "$ROOT"; OUT=gpurun_out/r6attnpf; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_transformer_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do for v in 1 0; do
  DTFX_ATTN_BWD_PF=$v timeout -k 10 120 python tools/probes/attn_one.py 40 > $OUT/attn_pf${v}_$r.json 2>&1 || { tail -5 $OUT/attn_pf${v}_$r.json; exit 1; }
  echo "attn pf=$v $r $(tail -1 $OUT/attn_pf${v}_$r.json)"
done; done
for r in 1 2 3; do for v in 1 0; do
  DTFX_ATTN_BWD_PF=$v timeout -k 10 200 python bench.py --model bert > $OUT/bert_pf${v}_$r.json 2>&1 || { tail -5 $OUT/bert_pf${v}_$r.json; exit 1; }
  echo "bert pf=$v $r $(tail -1 $OUT/bert_pf${v}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
}

exp_dp_ta8() {
# Round 6: BERT-base's data-parallel shape (tools/probes/dp_sim.py, simulated world 8) with the
# weight gradients on the 8-phase tile (DTFX_GEMM_TA8=1) against the 128x128 split-K default:
# in DP mode the weight gradients run on a side stream, where the 128x128 blocks (64 KB of LDS,
# two per CU) keep the data gradients' 8-phase blocks (128 KB) off those CUs.  Separate
# processes (the switch is read once), interleaved.
cd "$ROOT"; OUT=gpurun_out/r6dpta8; mkdir -p $OUT
for r in 1 2; do for v in 0 1; do
  DTFX_GEMM_TA8=$v timeout -k 10 500 python tools/probes/dp_sim.py --model bert --variants 1gpu,dp \
    --steps 10 --rounds 2 > $OUT/dp_ta8${v}_$r.json 2> $OUT/dp_ta8${v}_$r.err || { tail -20 $OUT/dp_ta8${v}_$r.err; exit 1; }
  echo "ta8=$v $r $(python -c "import json;d=json.load(open('$OUT/dp_ta8${v}_$r.json'))['ms_per_step'];print({k:(v['median'],v['vs_1gpu_pct']) for k,v in d.items()})")"
done; done
}

exp_ta8_ffn() {
# Round 6: BERT-base with only the FFN weight gradients on the 8-phase tile (DTFX_GEMM_TA8=2)
# against the 128x128 split-K default (=0), interleaved; the bf16 / BERT GPU tests first.
cd "$ROOT"; OUT=gpurun_out/r6ta8ffn; mkdir -p $OUT
DTFX_GEMM_TA8=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_bert_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do for v in 2 0; do
  DTFX_GEMM_TA8=$v timeout -k 10 200 python bench.py --model bert > $OUT/bert_ta8${v}_$r.json 2>&1 || { tail -5 $OUT/bert_ta8${v}_$r.json; exit 1; }
  echo "bert ta8=$v $r $(tail -1 $OUT/bert_ta8${v}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
}

case "${1:-}" in
  flush|pers|resnet_zero1|resnet_fold|attn_rp|k20_env|probe|attn_swz|resnet_wt|mlp_plan|zero_ranges|engines|attn_pf|dp_ta8|ta8_ffn) exp_"$1" ;;
  *) echo "usage: $0 {flush|pers|resnet_zero1|resnet_fold|attn_rp|k20_env|probe|attn_swz|resnet_wt|mlp_plan|zero_ranges|engines|attn_pf|dp_ta8|ta8_ffn}" >&2; exit 2 ;;
esac
