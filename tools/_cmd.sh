K="hub or spmm" bash tools/gpu_check.sh testsk && \
PTAG=_cfg2 BENCH_ARGS="--no-layer --no-cpu-reference" bash tools/gpu_check.sh prof pmc && \
PTAG=_ns BENCH_ARGS="--workload ns --no-layer --no-cpu-reference" bash tools/gpu_check.sh prof pmc && \
bash tools/gpu_check.sh bench bench_ns
