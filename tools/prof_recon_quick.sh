# k_recon kernels' durations (rocprofv3 kernel trace of the 8-frame batched decode driver).
# Usage: bash tools/prof_recon_quick.sh TAG [stream]
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
TAG=${1:-rq}; S=${2:-k4_low}
mkdir -p gpurun_out/$TAG
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/trace -o run -- python3 tools/recon_batch.py $S 8 5 > /dev/null 2> gpurun_out/$TAG/trace.err || { echo TRACE_FAIL; tail -20 gpurun_out/$TAG/trace.err; exit 1; }
python3 - "$TAG" <<'PY'
import csv, glob, sys
for f in glob.glob("gpurun_out/%s/trace/**/*kernel_stats.csv" % sys.argv[1], recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"].split("(")[0]
        if "recon" in n or "prep" in n or "deblock" in n:
            print("%-24s calls %6s avg %10.2f us  min %10.2f  max %10.2f" % (n, r["Calls"], float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3, float(r["MaxNs"]) / 1e3))
PY
