set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread tests/test_gpu_encoder_rd.py -k "hierarchical or gives_up" > gpurun_out/r03a_hdb.log 2>&1
