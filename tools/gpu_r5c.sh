# round-5 GPU pass: training / GAT / sampler tests, the default bench line, a kernel trace of the
# 3-launch sampler; a failing GPU step ends the script
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_training_gpu.py tests/test_gat_gpu.py tests/test_sampler_gpu.py -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread > gpurun_out/r5c_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5c_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python3 -u bench.py > gpurun_out/r5c_bench.json 2> gpurun_out/r5c_bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/r5c_sample -o run -- \
  python3 -u tools/sample_probe.py --reps 10 > gpurun_out/r5c_sample_prof.log 2>&1
find gpurun_out/prof/r5c_sample -type f ! -name '*kernel_stats.csv' -delete 2>/dev/null
exit 0
