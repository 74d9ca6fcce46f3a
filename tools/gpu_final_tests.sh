# round-end GPU check: the whole -m gpu suite (one process), smoke(), the default bench line;
# stops at a failure
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/final_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/final_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/final_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err
