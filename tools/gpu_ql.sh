# A/B of the encoder queue's priority levels (TE_QLEVELS variant library in var/) at the bench's workload
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/$1
THOR_AMD_LIB=var/lib_ql4.so timeout -k 10 300 python3 tools/seq_speed.py 240 batch/1 2 > gpurun_out/$1/ql4.txt 2>&1 || { tail gpurun_out/$1/ql4.txt; exit 1; }
grep mode gpurun_out/$1/ql4.txt
timeout -k 10 300 python3 tools/seq_speed.py 240 batch/1 2 > gpurun_out/$1/ql1.txt 2>&1 || { tail gpurun_out/$1/ql1.txt; exit 1; }
grep mode gpurun_out/$1/ql1.txt
