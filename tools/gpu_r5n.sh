# round-5 GPU pass n: the cfg3 GAT training step with er recomputed / gathered, alternated on one box
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python3 -u tools/train_step_probe.py --model gat --steps 20 >> gpurun_out/r5n_train_gat.log 2>&1 && \
  timeout -k 10 300 python3 -u tools/train_step_probe.py --model gat --steps 20 --er-gather >> gpurun_out/r5n_train_gat_gather.log 2>&1 || exit 1
done
timeout -k 10 300 python3 -u tools/gat_bwd_probe.py --reps 15 --short 8 > gpurun_out/r5n_gat_bwd_probe.log 2>&1
