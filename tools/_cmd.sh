set -o pipefail
export PYTHONUNBUFFERED=1
bash tools/profile_workload.sh r02z_cfg2 || exit $?
bash tools/profile_workload.sh r02z_ns --workload ns || exit $?
bash tools/profile_workload.sh r02z_cfg5 --workload cfg5 || exit $?
