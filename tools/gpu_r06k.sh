# Round 6k: final full GPU suite + smoke + default bench at HEAD
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r06k
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 1100 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], d['bit_exact'], r['avg_launch_us'], r['frac'], r['path']['frac'], r['path']['avg_us']);print(d['config']['enc_batch_frame_ms']);print(d.get('config3_encoder'));print(d.get('config5_encoder'));print(d.get('cpu_baseline'))"
