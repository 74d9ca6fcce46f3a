mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/xcd_ab.py --workload cfg2 --ks 262144 --degs 96,128,160,192 --chunks 64,128,256 --rounds 5 > gpurun_out/xcd_fine_cfg2.log 2>&1 && \
timeout -k 10 500 python -u tools/xcd_ab.py --workload ns --ks 262144 --degs 96,128,192 --chunks 64,128,256 --rounds 3 > gpurun_out/xcd_fine_ns.log 2>&1
