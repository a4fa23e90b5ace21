set -o pipefail
cd /root/repo
THOR_BENCH_RF_EARLY=1 timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04g_bench.json 2> gpurun_out/r04g_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r04g_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r04g_bench.json'));print(d['value'],d['ms_per_step'],d['bit_exact'],d['roofline']['avg_launch_us'],d['roofline'].get('avg_launch_us_before_steps'),d['roofline']['frac'])"
