OUT=gpurun_out/r01g bash tools/gpu_check.sh tests smoke bench bench_ns bench_gat bench_sage && \
timeout -k 10 900 python bench.py --workload cfg5 --steps 10 --warmup 3 > gpurun_out/r01g/bench_cfg5.log 2>&1 && tail -1 gpurun_out/r01g/bench_cfg5.log | cut -c1-300
