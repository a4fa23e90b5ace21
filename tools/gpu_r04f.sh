set -o pipefail
cd /root/repo
bash tools/prof_recon.sh r04f && python3 tools/pmc_kernel.py gpurun_out/r04f > gpurun_out/r04f/pmc.txt && cat gpurun_out/r04f/pmc.txt
