# round-6 GPU session: training / GAT tests, gemm_tn A/B, training-step probes, SpMM replay,
# cfg2 + cfg3 bench lines
set -o pipefail
mkdir -p gpurun_out/r6d
timeout -k 10 700 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_training_gpu.py tests/test_gat_gpu.py tests/test_fullsize_gpu.py -k "gemm_tn or training or gat" -p no:cacheprovider > gpurun_out/r6d/pytest.log 2>&1
rc=$?; grep -E "order, dropout|passed|failed|Error" gpurun_out/r6d/pytest.log | tail -12
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/gemm_tn_ab.py --reps 20 > gpurun_out/r6d/gemm_tn_ab.log 2>&1 || exit $?
timeout -k 10 200 python tools/spmm_replay.py --workload cfg2 > gpurun_out/r6d/replay_cfg2.log 2>&1 || exit $?
timeout -k 10 300 python tools/spmm_replay.py --workload ns --reps 10 > gpurun_out/r6d/replay_ns.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload cfg2 --steps 20 --warmup 5 > gpurun_out/r6d/bench_cfg2.json 2> gpurun_out/r6d/bench_cfg2.log || exit $?
timeout -k 10 300 python bench.py --workload cfg3 --steps 20 --warmup 5 > gpurun_out/r6d/bench_cfg3.json 2> gpurun_out/r6d/bench_cfg3.log || exit $?
python -c "
import json
for f in ('cfg2','cfg3'):
    d=json.load(open('gpurun_out/r6d/bench_%s.json'%f)); print(f, d['ms_per_step'], d.get('train_gcn_cfg2') or d.get('train_gat_cfg3'))"
