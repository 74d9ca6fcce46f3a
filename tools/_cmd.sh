set -o pipefail
O=gpurun_out/r02z; mkdir -p $O; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_spmm_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "xcd or rmat_1m" > $O/pytest_order.log 2>&1 || exit $?
timeout -k 10 300 python tools/xcd_ab.py --workload cfg2 --ks 262144 --degs 128 > $O/xcd_ab_order_cfg2.log 2>&1 || exit $?
timeout -k 10 400 python tools/xcd_ab.py --workload ns --ks 262144 --degs 128 > $O/xcd_ab_order_ns.log 2>&1 || exit $?
