# Round 5a: host-built slow list (no CAS in k_frame_prep) + encoder call-frame cuts (inline I-frame mode
# decision, final encode without a call): decode parity, isolated prep/recon timing, encoder A/B + parity, bench
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r05a
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_streams.py tests/test_gpu_recon.py tests/test_synth_frames.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_dec.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_dec.log; exit 1; }
tail -1 $OUT/pytest_dec.log
for s in k4_low k4_med; do timeout -k 10 120 python3 tools/recon_batch.py $s 8 10 --time > $OUT/time_$s.txt 2>&1 || { echo TIME_FAIL; tail $OUT/time_$s.txt; exit 1; }; cat $OUT/time_$s.txt; done
for V in PRE A PRE A; do
  if [ $V = A ]; then LIBP=thor_amd/libthor_amd.so; else LIBP=var/lib_$V.so; fi
  THOR_AMD_LIB=$LIBP timeout -k 10 170 python3 tools/enc_speed.py --name k4_low --batch 240 --frames 2 > $OUT/enc_$V.txt 2>&1 || { tail -20 $OUT/enc_$V.txt; exit 1; }
  echo "$V $(tail -1 $OUT/enc_$V.txt)"
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_encoder_rd.py > $OUT/pytest_enc.log 2>&1 || { echo PYTEST_ENC_FAIL; tail -30 $OUT/pytest_enc.log; exit 1; }
tail -1 $OUT/pytest_enc.log
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-legs > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], d['bit_exact'], r['avg_launch_us'], r['frac'], r['path']);print(d['config']['stage_ms_per_stream_pass'], d['config']['enc_batch_frame_ms'])"
