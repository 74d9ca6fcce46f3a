O=gpurun_out/r01j
OUT=$O bash tools/gpu_check.sh tests smoke bench bench_ns bench_gat bench_sage
