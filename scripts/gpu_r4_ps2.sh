# async-PS cluster after the ps reply-buffer reuse (two rounds each, one box)
set -o pipefail
mkdir -p gpurun_out/ps2
for r in 1 2; do
  timeout -k 10 200 python tools/bench_ps_async.py --num_workers 2 --steps 40000 > gpurun_out/ps2/w2_$r.json 2>/dev/null || exit 1
  timeout -k 10 200 python tools/bench_ps_async.py --num_workers 8 --steps 40000 > gpurun_out/ps2/w8_$r.json 2>/dev/null || exit 1
done
nproc > gpurun_out/ps2/nproc.txt
echo done
