set -o pipefail
O=gpurun_out/r02zf; mkdir -p $O; export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload cfg3 > $O/bench_gat.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --workload cfg4 > $O/bench_sage.log 2>&1 || exit $?
