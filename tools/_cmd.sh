mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/transform_ab.py --variants tf_base,tf_stage > gpurun_out/tf_stage_ab.log 2>&1
