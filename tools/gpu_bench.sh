# bench.py as the driver runs it, then its rocprofv3 kernel stats (one timed step).
# Usage: bash tools/gpu_bench.sh TAG [extra bench args]
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-bench}; shift
timeout -k 10 600 python -u bench.py "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
tail -c 3000 gpurun_out/${TAG}_bench.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-legs "$@" > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err || { echo PROF_FAIL; tail -20 gpurun_out/${TAG}_prof.err; exit 1; }
find gpurun_out/${TAG}_prof -name '*stats.csv'
