# Round 5q: encoder pipelining (begin/end) + early-skip cost re-use: encoder parity, then the bench (no legs)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r05q
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_encoder_rd.py -k "not hdb16" > $OUT/pytest_enc.log 2>&1 || { echo PYTEST_ENC_FAIL; tail -30 $OUT/pytest_enc.log; exit 1; }
tail -1 $OUT/pytest_enc.log
timeout -k 10 400 python bench.py --no-legs --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], d['bit_exact'], r['avg_launch_us'], r['frac'], r['path']['frac']);print(d['config']['enc_batch_frame_ms'], d['config']['pipe_timeline_last_step'])"
