set -o pipefail
O=gpurun_out/r02zf; mkdir -p $O; export PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py > $O/bench2.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --workload ns --no-cpu-reference > $O/bench_ns.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --workload cfg5 --no-cpu-reference > $O/bench_cfg5.log 2>&1 || exit $?
