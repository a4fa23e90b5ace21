# Round 5a: host-built slow list (no CAS in k_frame_prep): decode parity, isolated prep/recon timing, trace, bench
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r05a
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_streams.py tests/test_gpu_recon.py tests/test_synth_frames.py tests/test_gpu_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for s in k4_low k4_med; do timeout -k 10 120 python3 tools/recon_batch.py $s 8 10 --time > $OUT/time_$s.txt 2>&1 || { echo TIME_FAIL; tail $OUT/time_$s.txt; exit 1; }; cat $OUT/time_$s.txt; done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 tools/recon_batch.py k4_low 8 3 > /dev/null 2> $OUT/trace.err || { echo TRACE_FAIL; tail -20 $OUT/trace.err; exit 1; }
find $OUT/trace -name '*stats*' | head
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-legs > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], d['bit_exact'], r['avg_launch_us'], r['frac'], r['path']);print(d['config']['stage_ms_per_stream_pass'], d['config']['enc_batch_frame_ms'])"
