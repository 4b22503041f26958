timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py tests/test_xgmi_sim_gpu.py tests/test_xgmi_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2
for i in 1 2; do
  timeout -k 10 100 python bench.py 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('K=20000', d['value'], d['ms_per_step']*1000, d['final_loss'])"
  timeout -k 10 100 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('K=20', d['value'], d['ms_per_step']*1000)"
done
mkdir -p gpurun_out/tr
timeout -k 10 120 python tools/probes/mlp_pipelined_trace.py > gpurun_out/tr/ks28_head2.json 2>/dev/null
python -c "import json; d=json.load(open('gpurun_out/tr/ks28_head2.json')); print(d['untraced_us_per_step'], json.dumps(d['traced_step_replays'][-1]))"
