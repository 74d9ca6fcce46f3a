set -o pipefail
O=gpurun_out/r02z; mkdir -p $O; export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/xcd_ab.py --op gat --workload cfg2 --feat 64 --ks 131072,262144 --degs 512,1024,2048 --chunks 128,384 > $O/xcd_ab_gat_cfg3b.log 2>&1 || exit $?
