set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider -k "hub or spmm or gat or distributed or fullsize" --timeout 300 --timeout-method thread > gpurun_out/pytest_hub.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 400 python -u bench.py --workload ns --no-cpu-baseline --no-layer > gpurun_out/bench_ns_quick.log 2>&1
