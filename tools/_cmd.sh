set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_spmm_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_tf.log 2>&1
timeout -k 10 300 python -u tools/transform_ab.py > gpurun_out/transform_ab.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_tf.log 2>&1
