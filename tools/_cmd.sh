bash tools/gpu_check.sh prof pmc && \
BENCH_ARGS="--workload ns" OUT=gpurun_out/ns bash tools/gpu_check.sh pmc && \
bash tools/gpu_check.sh bench_ns bench_sage
