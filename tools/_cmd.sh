mkdir -p gpurun_out
{
python -c "
import torch, time
p = torch.cuda.get_device_properties(0); print(p)
x = torch.empty(2**28, device='cuda'); y = torch.empty_like(x)
for _ in range(3): y.copy_(x)
torch.cuda.synchronize(); t=time.time()
for _ in range(20): y.copy_(x)
torch.cuda.synchronize(); dt=(time.time()-t)/20; print('copy 1 GiB -> GB/s', 2*2**30/dt/1e9)
"
rocm-smi --showcomputepartition --showmemorypartition --showclocks 2>&1 | head -40
} > gpurun_out/boxinfo.log 2>&1
