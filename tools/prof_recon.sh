# k_recon evidence on its bench form (8-frame batched launches, tools/recon_batch.py), run on the GPU box:
#   hipEvent timing, kernel trace + stats, SQ counter passes, HBM bytes (FETCH_SIZE, WRITE_SIZE) passes.
# Usage: bash tools/prof_recon.sh TAG
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
TAG=${1:-recon}
OUT=gpurun_out/$TAG
mkdir -p $OUT
D="python3 tools/recon_batch.py k4_low 8 3"
P="python3 tools/recon_probe.py k4_low"
timeout -k 10 120 python3 tools/recon_batch.py k4_low 8 10 --time > $OUT/time.txt 2>&1 || { echo TIME_FAIL; tail $OUT/time.txt; exit 1; }
cat $OUT/time.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- $D > /dev/null 2> $OUT/trace.err || { echo TRACE_FAIL; tail -20 $OUT/trace.err; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d $OUT/sq1 -o run -- $D > /dev/null 2> $OUT/sq1.err || { echo SQ1_FAIL; tail -20 $OUT/sq1.err; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-trace -d $OUT/sq2 -o run -- $D > /dev/null 2> $OUT/sq2.err || { echo SQ2_FAIL; tail -20 $OUT/sq2.err; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run -- $D > /dev/null 2> $OUT/fetch.err || { echo FETCH_FAIL; tail -20 $OUT/fetch.err; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run -- $D > /dev/null 2> $OUT/write.err || { echo WRITE_FAIL; tail -20 $OUT/write.err; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $OUT/ta -o run -- $D > /dev/null 2> $OUT/ta.err || echo TA_FAIL
timeout -k 10 120 $P > $OUT/probe.txt 2>&1 || { echo PROBE_FAIL; tail $OUT/probe.txt; exit 1; }
find $OUT -name '*.csv' | head -40
