# Round 6l (round-end evidence): rocprof evidence at HEAD -- k_recon on its 8-frame launch (timing, trace, SQ, FETCH/WRITE, TA),
# then the bench under rocprofv3 (kernel trace + stats) and the decoder FETCH/WRITE passes
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
bash tools/prof_recon.sh r06l_recon || exit 1
python3 tools/pmc_kernel.py gpurun_out/r06l_recon k_recon > gpurun_out/r06l_recon/pmc.txt || exit 1
python3 tools/pmc_kernel.py gpurun_out/r06l_recon k_frame_prep > gpurun_out/r06l_recon/pmc_prep.txt || exit 1
bash tools/profile_round.sh || exit 1
