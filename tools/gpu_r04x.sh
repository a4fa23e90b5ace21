# Round-4 closing pass: encoder A/B + encoder tests, smoke, bench under rocprofv3 (profile_round.sh).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
VARS="${VARS:-PRE A PRE A}" bash tools/gpu_r04s.sh || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04x_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/r04x_smoke.log; exit 1; }
tail -1 gpurun_out/r04x_smoke.log
[ -n "$NO_PROF" ] || bash tools/profile_round.sh || exit 1
