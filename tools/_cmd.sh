set -e
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_graph_build_gpu.py tests/test_distributed_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_feat.log 2>&1
