# k_recon 2-units-per-block A/B + parity, encoder A/B (search_intra8) + encoder tests.
set -o pipefail
cd /root/repo
VARS="A U2 A U2" PVARS="U2" bash tools/gpu_var.sh || exit 1
VARS="PRE A PRE A" bash tools/gpu_r04s.sh || exit 1
