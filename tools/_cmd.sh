mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gat_gpu.py tests/test_han_sagepy_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t_gat.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload cfg3 --steps 20 --warmup 5 > gpurun_out/bench_gat.log 2>&1
