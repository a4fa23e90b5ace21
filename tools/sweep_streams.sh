# bench.py over (streams, groups) pairs on the GPU box: sweep_streams.sh "15 3" "24 3" ...
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/sweep
for sg in "$@"; do
  set -- $sg
  timeout -k 10 150 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --streams $1 --groups $2 > gpurun_out/sweep/sg_$1_$2.json 2> gpurun_out/sweep/sg_$1_$2.err || { echo FAIL $sg; tail -5 gpurun_out/sweep/sg_$1_$2.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sweep/sg_$1_$2.json'));r=d['roofline'];print('streams/groups', '$1/$2', d['value'], d['ms_per_step'], r['frames_per_launch'], r['avg_launch_us'], r['frac'], d['bit_exact'])"
done
