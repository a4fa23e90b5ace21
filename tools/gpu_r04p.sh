# Round-4 profiles: k_recon on its 8-frame launch (prof_recon.sh: trace + SQ + FETCH/WRITE + TA passes),
# then the bench under rocprofv3 (profile_round.sh: kernel trace + stats, decoder FETCH/WRITE passes).
set -o pipefail
cd /root/repo
bash tools/prof_recon.sh r04p_recon || exit 1
bash tools/profile_round.sh || exit 1
