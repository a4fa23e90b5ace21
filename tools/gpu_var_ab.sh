# A/B of an encoder variant library (var/lib_$2.so) against the product build at the bench's workload
# usage: bash tools/gpu_var_ab.sh TAG VARIANT
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/$1
THOR_AMD_LIB=var/lib_$2.so timeout -k 10 300 python3 tools/seq_speed.py 240 batch/1 2 > gpurun_out/$1/$2.txt 2>&1 || { tail gpurun_out/$1/$2.txt; exit 1; }
grep mode gpurun_out/$1/$2.txt | cut -c1-330
timeout -k 10 300 python3 tools/seq_speed.py 240 batch/1 2 > gpurun_out/$1/product.txt 2>&1 || { tail gpurun_out/$1/product.txt; exit 1; }
grep mode gpurun_out/$1/product.txt | cut -c1-330
