# Instruction-cache counters of the encoder (k_enc_rows) on its I frame: 64 streams of hd_low.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r04l
mkdir -p $O
D="python3 tools/enc_speed.py --name hd_low --batch 64 --frames 1"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -d $O/ic -o run -- $D > /dev/null 2> $O/ic.err || { echo IC_FAIL; tail -20 $O/ic.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH_LEVEL SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_SMEM SQ_LEVEL_WAVES SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA --kernel-trace -d $O/lv -o run -- $D > /dev/null 2> $O/lv.err || { echo LV_FAIL; tail -20 $O/lv.err; exit 1; }
echo done
