# H2D A/B: the bench's raw-frame copies (12.4 MB pinned -> HBM) via torch copy_ and
# via hipMemcpyAsync, each under a kernel trace (blit kernels vs the copy engines) -- gpurun_out/$1
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 120 python3 tools/h2d_probe.py 64 > $OUT/probe_default.txt 2>&1 && cat $OUT/probe_default.txt &&
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $OUT/prof -o h2d -- python3 tools/h2d_probe.py 64 > $OUT/probe_prof.txt 2>&1 && tail -3 $OUT/probe_prof.txt &&
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \; &&
find $OUT/prof -name "*memory_copy_stats.csv" -exec cp {} $OUT/copy_stats.csv \; ;
cat $OUT/kernel_stats.csv 2>/dev/null | head -5; cat $OUT/copy_stats.csv 2>/dev/null | head -5
