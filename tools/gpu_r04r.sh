# CU-mask experiment: bench value and in-bench decode kernel times with the encoder kept off N of every 32 CUs.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r04r
mkdir -p $O
for N in ${NS:-0 1 2}; do
  timeout -k 10 170 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-legs --enc-cu-exclude $N > $O/bench_x$N.json 2> $O/bench_x$N.err || { echo BENCH_FAIL $N; tail -20 $O/bench_x$N.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_x$N.json'));print('exclude $N', d['value'], d['ms_per_step'], d['config']['pipe_timeline_last_step'])"
done
for N in ${PNS:-0 2}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_x$N -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-legs --enc-cu-exclude $N > $O/trace_x$N.json 2> $O/trace_x$N.err || { echo TRACE_FAIL $N; tail -20 $O/trace_x$N.err; exit 1; }
done
echo done
