set -o pipefail
cd /root/repo
bash tools/gpu_suite.sh r04e || exit 1
timeout -k 10 400 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r04e_bench.json 2> gpurun_out/r04e_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r04e_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r04e_bench.json'));print(d['value'],d['ms_per_step'],d['roofline'])"
