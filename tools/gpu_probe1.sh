#!/bin/bash
# First GPU probe: stock-PyTorch reference-equivalent ResNet-50 numbers + rocprof kernel breakdown.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 400 python bench.py --impl torch --channels-last 1 --steps 20 --warmup 10 > gpurun_out/torch_cl_b256.log 2>&1 && \
timeout -k 10 300 python bench.py --impl torch --channels-last 0 --steps 20 --warmup 10 > gpurun_out/torch_nchw_b256.log 2>&1 && \
timeout -k 10 300 python -c "
import torch,time
for n in (4096,8192):
  a=torch.randn(n,n,device='cuda',dtype=torch.bfloat16); b=torch.randn(n,n,device='cuda',dtype=torch.bfloat16)
  for _ in range(3): a@b
  torch.cuda.synchronize(); t=time.time()
  for _ in range(20): a@b
  torch.cuda.synchronize(); dt=(time.time()-t)/20
  print('matmul',n,2*n**3/dt/1e12,'TF')
x=torch.empty(1<<28,device='cuda',dtype=torch.float32)
torch.cuda.synchronize(); t=time.time()
for _ in range(20): y=x.clone()
torch.cuda.synchronize(); dt=(time.time()-t)/20
print('copy GB/s', 2*x.numel()*4/dt/1e9)
" > gpurun_out/calib.log 2>&1 && \
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_torch -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --impl torch --channels-last 1 --steps 5 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_torch.log 2>&1
