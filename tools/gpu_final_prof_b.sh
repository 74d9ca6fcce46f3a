# round-end profiles, part b: cfg3 and cfg4, then the default bench line
set -eo pipefail
export TAG=r5z SQ=1 WORKLOADS="cfg3 cfg4"
bash tools/profile_round.sh > gpurun_out/profile_round_r5z_b.log 2>&1
