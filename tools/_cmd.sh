set -o pipefail
O=gpurun_out/r02z; mkdir -p $O; export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_sampler_gpu.py tests/test_sage_gpu.py tests/test_han_sagepy_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_frontier.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --workload cfg4 --no-cpu-baseline > $O/bench_sage_frontier.log 2>&1 || exit $?
