# round-5 GPU pass d: the two-pass GAT backward (tests, cfg3 comparison), the sampler tests
# after the one-allocation change, the default bench line; a failing GPU step ends the script
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gat_gpu.py tests/test_sampler_gpu.py tests/test_training_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5d_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r5d_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py > gpurun_out/r5d_bench.json 2> gpurun_out/r5d_bench.err
