set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/gat_ab.py --variants base,gs4,gs8 --rounds 8 > gpurun_out/gat_gs_slow.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_dist2.log 2>&1
