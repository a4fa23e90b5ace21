# quick GPU check: stream parity tests + a short bench (no CPU baseline)
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_streams.py tests/test_synth_frames.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/quick_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/quick_pytest.log; exit 1; }
tail -2 gpurun_out/quick_pytest.log
timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/quick_bench.json 2> gpurun_out/quick_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/quick_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/quick_bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
