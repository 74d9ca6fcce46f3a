set -o pipefail
O=gpurun_out/r02z; mkdir -p $O; export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --workload ns > $O/bench_ns.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --workload cfg5 --no-cpu-reference > $O/bench_cfg5.log 2>&1 || exit $?
