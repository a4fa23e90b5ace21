set -o pipefail
cd /root/repo
bash tools/prof_recon.sh r04b && python3 tools/pmc_kernel.py gpurun_out/r04b > gpurun_out/r04b/pmc.txt && cat gpurun_out/r04b/pmc.txt && cat gpurun_out/r04b/probe.txt
