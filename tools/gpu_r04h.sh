set -o pipefail
cd /root/repo
for X in 0 120 232; do
  echo "== RB_EXTRA=$X"; RB_EXTRA=$X timeout -k 10 200 python3 tools/recon_batch.py k4_low 8 10 --time > gpurun_out/rbx.log 2>&1 || { tail -5 gpurun_out/rbx.log; exit 1; }
  grep avg gpurun_out/rbx.log
done
THOR_BENCH_RF_EARLY=1 timeout -k 10 300 python bench.py --streams 16 --steps 2 --warmup 1 --no-cpu-baseline --no-legs > gpurun_out/r04h_bench.json 2> gpurun_out/r04h_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r04h_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r04h_bench.json'));print('bench16', d['value'],d['roofline']['avg_launch_us'],d['roofline'].get('avg_launch_us_before_steps'))"
