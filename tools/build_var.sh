# build a k_recon / encoder variant library with the product's flags plus extra ones:
#   tools/build_var.sh NAME -DMACRO=V ...
set -e
cd /root/repo
mkdir -p var
N=$1; shift
FLAGS=$(python3 -c "import sys; sys.path.insert(0, '.'); from thor_amd.build import FLAGS; print(' '.join(f for f in FLAGS if f != '-DRECON_WPE=5'))")
/opt/rocm/bin/hipcc $FLAGS -w -DRECON_WPE=5 "$@" -o var/lib_$N.so thor_amd/csrc/libthor_amd.hip
