K=gat bash tools/gpu_check.sh testsk bench_gat && \
AB_ARGS="--variants 0,8,9 --hot-mib 64 --seg-lens 64,192,256" bash tools/gpu_check.sh ab && \
AB_ARGS="--variants 9 --hot-mib 160" OUT=gpurun_out/h160 bash tools/gpu_check.sh ab && \
AB_WL=ns AB_ARGS="--variants 0,8,9 --hot-mib 128 --seg-len 256" OUT=gpurun_out/ns bash tools/gpu_check.sh ab && \
AB_WL=ns AB_ARGS="--variants 9 --hot-mib 200 --seg-len 256" OUT=gpurun_out/ns200 bash tools/gpu_check.sh ab
