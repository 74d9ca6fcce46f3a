mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u tools/project_ab.py --variants base,nomfma,nowh,g2,g2_512,blds,g512 > gpurun_out/proj_ab.log 2>&1 && \
timeout -k 10 200 python -u tools/project_ab.py --variants g2,base,g2_512,blds,g512 >> gpurun_out/proj_ab.log 2>&1
