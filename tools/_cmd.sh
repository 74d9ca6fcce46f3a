set -o pipefail
O=gpurun_out/r02z; mkdir -p $O; export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_sage_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_sage_fused.log 2>&1 || exit $?
timeout -k 10 300 python tools/sage_layer_ab.py > $O/sage_layer_ab.log 2>&1 || exit $?
