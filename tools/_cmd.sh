set -e
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_spmm_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k xcd > gpurun_out/t_xcd.log 2>&1
timeout -k 10 300 python -u tools/xcd_ab.py --workload cfg2 --ks 262144 --degs 64,128 --item-rows 0,32768,65536,131072 > gpurun_out/xcd_ik_cfg2.log 2>&1
timeout -k 10 400 python -u tools/xcd_ab.py --workload ns --ks 262144 --degs 128 --item-rows 0,32768,65536,131072 --rounds 4 > gpurun_out/xcd_ik_ns.log 2>&1
