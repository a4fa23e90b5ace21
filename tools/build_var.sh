# build a k_recon / encoder variant library: tools/build_var.sh NAME -DMACRO=V ...
set -e
cd /root/repo
mkdir -p var
N=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -w -Xclang -target-feature -Xclang -dot6-insts -Xclang -target-feature -Xclang -dot4-insts "$@" -o var/lib_$N.so thor_amd/csrc/libthor_amd.hip
