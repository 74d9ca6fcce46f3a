# round-5 GPU pass j: the scan's flat prefix sum (sampler tests, probe, per-call kernel trace);
# the GAT aggregation without its er gathers (traffic probe variant) beside the default
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_sampler_gpu.py tests/test_sage_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5j_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r5j_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/sample_probe.py > gpurun_out/r5j_sample_probe.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof/r5j_sample -o run -- python3 -u tools/sample_probe.py > gpurun_out/r5j_sample_trace.log 2>&1 && \
timeout -k 10 300 python3 -u tools/gat_tasks_ab.py --reps 30 --libs noer > gpurun_out/r5j_gat_noer_ab.log 2>&1
rc=$?
find gpurun_out/prof/r5j_* -type f ! -name '*kernel_trace.csv' -delete 2>/dev/null
exit $rc
