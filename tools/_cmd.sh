mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u bench.py --workload ns --steps 20 --warmup 5 --no-cpu-reference > gpurun_out/bench_ns.log 2>&1 && \
timeout -k 10 500 python -u bench.py --workload cfg5 --steps 10 --warmup 3 --no-cpu-reference > gpurun_out/bench_cfg5.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload cfg4 --steps 20 --warmup 5 > gpurun_out/bench_sage.log 2>&1
