for v in 1 2; do
  for lim in default big; do
    if [ $lim = big ]; then export HSA_SCRATCH_SINGLE_LIMIT=8589934592; else unset HSA_SCRATCH_SINGLE_LIMIT; fi
    echo "== wpe $v scratch $lim" >> gpurun_out/r02n_speed.txt
    THOR_AMD_LIB=$PWD/thor_amd/libthor_amd_wpe$v.so timeout -k 10 200 python -u tools/enc_speed.py --batch 32 64 >> gpurun_out/r02n_speed.txt 2>&1 || exit 1
  done
done
