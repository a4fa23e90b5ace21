set -o pipefail
cd /root/repo
VARS="W5 P1 P2 P3" PVARS="" bash tools/gpu_var.sh || exit 1
cp var/lib_W5.so thor_amd/libthor_amd.so
bash tools/prof_recon.sh r04c && python3 tools/pmc_kernel.py gpurun_out/r04c > gpurun_out/r04c/pmc.txt && cat gpurun_out/r04c/pmc.txt && head -12 gpurun_out/r04c/probe.txt
