# round-5 GPU pass t: edge-head layout A/B with er recomputed
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/gat_tasks_ab.py --reps 40 --libs noeh,noeh+rec > gpurun_out/r5t_gat_ab.log 2>&1
