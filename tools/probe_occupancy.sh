# k_recon phase stamps (tools/recon_probe.py) under occupancy caps set by THOR_RECON_LDS_PAD
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/occ
for pad in "$@"; do
  THOR_RECON_LDS_PAD=$pad timeout -k 10 120 python tools/recon_probe.py k4_low > gpurun_out/occ/probe_$pad.txt 2>&1 || { echo FAIL $pad; tail -5 gpurun_out/occ/probe_$pad.txt; exit 1; }
  echo "pad $pad"; grep -m1 -A8 "frame 2" gpurun_out/occ/probe_$pad.txt | grep -v slowest | grep -v latest
done
