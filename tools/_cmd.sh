mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_distributed_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t_gat_staged2.log 2>&1
