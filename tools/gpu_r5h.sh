# round-5 GPU pass h: kernel traces of the sampler (per call) and of the cfg2 GCN / cfg3 GAT
# training steps; a failing GPU step ends the script
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof/r5h_sample -o run -- python3 -u tools/sample_probe.py > gpurun_out/r5h_sample.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/r5h_gcn -o run -- python3 -u tools/train_step_probe.py --model gcn > gpurun_out/r5h_gcn.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/r5h_gat -o run -- python3 -u tools/train_step_probe.py --model gat > gpurun_out/r5h_gat.log 2>&1
rc=$?
find gpurun_out/prof/r5h_* -type f ! -name '*kernel_stats.csv' ! -name '*kernel_trace.csv' -delete 2>/dev/null
exit $rc
