set -o pipefail
cd /root/repo
VARS="W5 D5 D1 W5 D5 D1" PVARS="D5" bash tools/gpu_var.sh
