set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gat_gpu.py tests/test_han_sagepy_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_pack.log 2>&1
timeout -k 10 300 python -u tools/gat_pack_ab.py > gpurun_out/gat_pack_ab.log 2>&1
