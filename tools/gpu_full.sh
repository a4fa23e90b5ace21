# Full GPU round on the box: pytest -m gpu, bench (with CPU baseline), then the
# rocprofv3 kernel-trace + FETCH/WRITE PMC passes (tools/profile_round.sh).
set -o pipefail
cd /root/repo
bash tools/gpu_round.sh || exit 1
bash tools/profile_round.sh || exit 1
