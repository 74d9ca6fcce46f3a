O=gpurun_out/r01i
OUT=$O bash tools/gpu_check.sh tests smoke bench bench_ns bench_gat bench_sage && \
PTAG=_cfg3 OUT=$O BENCH_ARGS="--workload cfg3" bash tools/gpu_check.sh prof pmc && \
PTAG=_cfg4 OUT=$O BENCH_ARGS="--workload cfg4" bash tools/gpu_check.sh prof pmc && \
PTAG=_cfg2 OUT=$O BENCH_ARGS="--no-layer --no-cpu-reference" bash tools/gpu_check.sh prof && \
timeout -k 10 900 python bench.py --workload cfg5 --steps 10 --warmup 3 > $O/bench_cfg5.log 2>&1 && \
OUT=$O bash tools/gpu_check.sh rehearse2
