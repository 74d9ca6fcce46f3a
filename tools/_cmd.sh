bash tools/gpu_check.sh tests && \
PTAG=_cfg3 BENCH_ARGS="--workload cfg3" bash tools/gpu_check.sh prof pmc && \
bash tools/gpu_check.sh bench_gat && \
step_cfg5() { timeout -k 10 900 python bench.py --workload cfg5 --steps 10 --warmup 3 > gpurun_out/bench_cfg5.log 2>&1; } && step_cfg5 && tail -2 gpurun_out/bench_cfg5.log
