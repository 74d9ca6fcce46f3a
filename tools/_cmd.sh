set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider -k "gat or han or spmm or hub" --timeout 300 --timeout-method thread > gpurun_out/pytest_gs.log 2>&1
timeout -k 10 300 python -u bench.py --workload cfg3 --no-cpu-baseline > gpurun_out/bench_gat_gs.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-layer > gpurun_out/bench_cfg2_gs.log 2>&1
