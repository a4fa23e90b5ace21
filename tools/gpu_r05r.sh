# Round 5r: k_recon residual prefetch A/B; the threaded multi-rank device-exchange tests (tests/fake_dist.py), then the full
# GPU suite at HEAD (encoder pipelining, fused early skip, frame image upload) + smoke
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r05r
mkdir -p $OUT
# k_recon A/B: residual lines prefetched into L2 at plan time (product) vs not (var/lib_NOPF.so)
for V in A NOPF A NOPF; do
  if [ $V = A ]; then LIBP=thor_amd/libthor_amd.so; else LIBP=var/lib_$V.so; fi
  THOR_AMD_LIB=$LIBP timeout -k 10 120 python3 tools/recon_batch.py k4_low 8 10 --time > $OUT/time_$V.txt 2>&1 || { echo TIME_FAIL; tail $OUT/time_$V.txt; exit 1; }
  echo "$V $(tail -2 $OUT/time_$V.txt | tr '\n' ' ')"
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py -x -v -k threads --timeout 120 --timeout-method thread > $OUT/pytest_threads.log 2>&1 || { echo THREADS_FAIL; tail -60 $OUT/pytest_threads.log; exit 1; }
tail -3 $OUT/pytest_threads.log
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
