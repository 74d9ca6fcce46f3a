set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/lib_ab.py --op sage --variants base,su2,su8,su16 --workload ns > gpurun_out/sage_u_ab.log 2>&1
