# round-5 GPU pass o: the GAT aggregation of this tree beside the pre-er-change kernels
# (variant library gatr5j) in one process
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/gat_tasks_ab.py --reps 40 --libs gatr5j > gpurun_out/r5o_gat_ab.log 2>&1
