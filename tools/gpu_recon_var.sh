# k_recon / k_frame_prep timing of variant libraries (var/lib_<name>.so) against the product build,
# the isolated 8-frame 4K P launches of tools/recon_batch.py.  usage: bash tools/gpu_recon_var.sh TAG NAME...
set -o pipefail
cd /root/repo
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for v in product "$@" product; do
  L=thor_amd/libthor_amd.so; [ $v = product ] || L=var/lib_$v.so
  THOR_AMD_LIB=$L timeout -k 10 120 python3 tools/recon_batch.py k4_low 8 10 --time > gpurun_out/$TAG/recon_$v.txt 2>&1 || exit 1
  echo "== $v"; head -2 gpurun_out/$TAG/recon_$v.txt
done
