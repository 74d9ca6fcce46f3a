# round-end default bench line on the committed tree (traffic files stamped with it)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u bench.py > gpurun_out/final_bench2.json 2> gpurun_out/final_bench2.err
