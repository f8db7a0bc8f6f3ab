#!/bin/bash
# TinyImageNet kernel stats with the side stream (default) and in order (DBX_OVERLAP_WGRAD=0): which main-chain
# kernels slow down beside the weight gradients
set -o pipefail
O=${1:-gpurun_out/tiny_stats}
mkdir -p $O
export TMPDIR=/tmp
for ov in def 0; do
  env $( [ $ov = def ] && echo DBX_PROFILE_DEFAULT=1 || echo DBX_OVERLAP_WGRAD=$ov ) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rp_ov$ov -o run -- python3 bench.py --preset resnet50_tiny_imagenet --steps 10 --warmup 4 > $O/ov$ov.log 2>&1 || { tail -20 $O/ov$ov.log; exit 1; }
  python3 tools/prof_top.py $(find $O/rp_ov$ov -name "run_kernel_stats.csv" | head -1) 14 80 > $O/top_ov$ov.txt 2>&1 || true
done
