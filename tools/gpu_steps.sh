# One gpurun call = a list of steps, each under its own time limit, stopping at
# the first failure; every output under gpurun_out/TAG/ (merged back by gpurun).
# Replaces the per-call tools/gpu_rNNx.sh scripts of rounds 3-5.
#
# Usage: bash tools/gpu_steps.sh TAG STEP [STEP ...]
#   pytest:EXPR           the -m gpu tests matching -k EXPR ("all": the whole suite)
#   smoke                 __graft_entry__.smoke()
#   recon:STREAM          tools/recon_batch.py STREAM 8 10 --time (k_frame_prep / k_recon per 8-frame launch)
#   bands:STREAM:WORLD    tools/band_split.py STREAM WORLD all (per-rank kernel time of the row split)
#   bandprof:STREAM:WORLD:RANK  the same for one rank under rocprofv3 --kernel-trace --stats
#   bench:ARGS            python bench.py ARGS (commas -> spaces)
#   profrecon             tools/prof_recon.sh TAG_recon (k_recon / k_frame_prep trace, SQ, FETCH / WRITE)
#   profbench             tools/profile_round.sh (bench kernel trace + decoder FETCH / WRITE)
#   encspeed:ARGS         tools/enc_speed.py ARGS (commas -> spaces)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
( while sleep 30; do date +%T >> $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}
  arg=${step#*:}
  [ "$arg" = "$step" ] && arg=""
  log=$OUT/$(printf %02d $n)_$kind.log
  echo "== step $n: $step" | tee -a $OUT/steps.txt
  case $kind in
    pytest)
      K=""; [ "$arg" != "all" ] && [ -n "$arg" ] && K="$arg"
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v -s --durations=15 --timeout 600 --timeout-method thread ${K:+-k "$K"} > $log 2>&1
      rc=$?; grep -E "passed|failed|error" $log | tail -2 ;;
    smoke)
      timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $log 2>&1; rc=$?; tail -1 $log ;;
    recon)
      timeout -k 10 150 python3 tools/recon_batch.py $arg 8 10 --time > $log 2>&1; rc=$?; cat $log ;;
    bands)
      IFS=: read s w <<< "$arg"
      timeout -k 10 300 python3 tools/band_split.py $s $w all > $log 2>&1; rc=$?; cat $log ;;
    bandprof)
      IFS=: read s w r <<< "$arg"
      timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/bandprof_${w}_${r} -o run -- python3 tools/band_split.py $s $w $r > $log 2>&1; rc=$?; tail -2 $log ;;
    bench)
      timeout -k 10 900 python bench.py ${arg//,/ } > $OUT/bench_$n.json 2> $log; rc=$?; tail -c 3000 $OUT/bench_$n.json ;;
    profrecon)
      timeout -k 10 900 bash tools/prof_recon.sh ${TAG}_recon > $log 2>&1; rc=$?; tail -5 $log ;;
    profbench)
      timeout -k 10 900 bash tools/profile_round.sh > $log 2>&1; rc=$?; tail -5 $log ;;
    encspeed)
      timeout -k 10 900 python3 tools/enc_speed.py ${arg//,/ } > $log 2>&1; rc=$?; tail -20 $log ;;
    *)
      echo "unknown step $step"; rc=2 ;;
  esac
  if [ $rc -ne 0 ]; then
    echo "STEP_FAIL $step rc=$rc"; tail -40 $log; exit 1
  fi
done
echo ALL_STEPS_OK
