# round-5 GPU pass q: MAX / MAXPOOL inference through the one-launch concat + MFMA layer
# (sage, sampler, C-ABI tests; cfg4 bench line with the aggregator variants)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_sage_gpu.py tests/test_sampler_gpu.py tests/test_capi.py tests/test_han_sagepy_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5q_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5q_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --workload cfg4 --steps 30 --warmup 5 --no-cpu-baseline --no-cpu-reference > gpurun_out/r5q_cfg4.json 2> gpurun_out/r5q_cfg4.log
