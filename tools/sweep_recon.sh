# k_recon tuning sweep on the GPU box: bench.py under each value of a
# THOR_RECON_* environment knob (usage: sweep_recon.sh VAR v1 v2 ...)
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/sweep
var=$1; shift
for w in "$@"; do
  env $var=$w timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sweep/$var.$w.json 2> gpurun_out/sweep/$var.$w.err || { echo FAIL $w; tail -5 gpurun_out/sweep/$var.$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sweep/$var.$w.json'));print('$var', $w, d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done
