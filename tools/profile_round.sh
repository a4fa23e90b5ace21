# rocprofv3 evidence for bench.py (run on the GPU box via gpurun).
#   pass 1: kernel trace + stats (per-kernel average durations)
#   pass 2/3: HBM bytes (FETCH_SIZE, WRITE_SIZE) in separate --pmc passes
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-legs --no-rows"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- $B > $OUT/trace_bench.json 2> $OUT/trace.err || { echo TRACE_FAIL; tail -20 $OUT/trace.err; exit 1; }
# PMC passes on the decoder alone (the encoder's persistent workers run for minutes with counters on):
# one 4K LDB-low frame per launch, frames in decode order I P P P P P P P
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run -- python3 tools/decode_frames.py k4_low 8 > /dev/null 2> $OUT/fetch.err || { echo FETCH_FAIL; tail -20 $OUT/fetch.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run -- python3 tools/decode_frames.py k4_low 8 > /dev/null 2> $OUT/write.err || { echo WRITE_FAIL; tail -20 $OUT/write.err; exit 1; }
find $OUT -name '*.csv' | head -50
