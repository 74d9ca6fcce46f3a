# round-end profiles of the final tree (stats, FETCH / WRITE / L2, SQ passes for every workload),
# then the default bench line; TAG names the round
set -eo pipefail
export TAG=${TAG:-r6f4} SQ=1
bash tools/profile_round.sh > gpurun_out/profile_round_${TAG}.log 2>&1
