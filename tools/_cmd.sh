set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_han_sagepy_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/han_t.log 2>&1
timeout -k 10 200 python -u tools/han_ab.py > gpurun_out/han_ab.log 2>&1
timeout -k 10 200 python -u tools/han_ab.py --n 20000 --deg 32 >> gpurun_out/han_ab.log 2>&1
timeout -k 10 200 python -u tools/han_ab.py --n 3025 --deg 40 --fin 1870 >> gpurun_out/han_ab.log 2>&1
