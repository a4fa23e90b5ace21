# Round 6d: the default bench (all legs, CPU baseline) with the SB scheduler
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r06d
mkdir -p $OUT
timeout -k 10 1100 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], d['bit_exact'], r['avg_launch_us'], r['frac'], r['path']['frac'], r['path']['avg_us']);print(d['config']['enc_batch_frame_ms']);print(d.get('config3_encoder'));print(d.get('config5_encoder'));print(d.get('cpu_baseline'))"
