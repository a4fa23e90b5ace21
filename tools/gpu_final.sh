# Round-end evidence on the box: the default bench line (legs, CPU baseline, rows), then the bench under
# rocprofv3 --kernel-trace --stats and the decoder FETCH / WRITE passes (tools/profile_round.sh).
# Usage: bash tools/gpu_final.sh TAG   (outputs under gpurun_out/TAG and gpurun_out/prof)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
TAG=${1:-final}
mkdir -p gpurun_out/$TAG
timeout -k 10 700 python bench.py --steps 5 --warmup 1 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/$TAG/bench.err; exit 1; }
tail -c 600 gpurun_out/$TAG/bench.json
[ -n "$WITH_PROFILE" ] || { echo FINAL_OK; exit 0; }
timeout -k 10 700 bash tools/profile_round.sh > gpurun_out/$TAG/profile.log 2>&1 || { echo PROFILE_FAIL; tail -20 gpurun_out/$TAG/profile.log; exit 1; }
echo FINAL_OK
