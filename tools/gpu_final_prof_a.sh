# round-end profiles, part a: cfg2 and the north star (stats, FETCH / WRITE / L2, SQ passes)
set -eo pipefail
export TAG=r5z SQ=1 NO_BENCH=1 WORKLOADS="cfg2 ns"
bash tools/profile_round.sh > gpurun_out/profile_round_r5z_a.log 2>&1
