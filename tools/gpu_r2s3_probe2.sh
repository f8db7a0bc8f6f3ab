#!/bin/bash
# PMC counters of the patch kernel vs the implicit GEMM on the 64-channel 3x3 convs.
set -o pipefail
mkdir -p gpurun_out/r2s3/probe2
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for c in "fwd3x3_64 patch" "dgrad3x3_64 patch" "fwd3x3_64 128,64,1"; do
  set -- $c
  tag=${1}_${2//,/x}
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $R/gpurun_out/r2s3/probe2/$tag/a -o run --output-format csv -- python3 $R/tools/conv_probe.py --case $1 --tile $2 --iters 2 > /dev/null 2>&1 || { echo "pmc a $tag failed"; exit 1; }
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR -d $R/gpurun_out/r2s3/probe2/$tag/b -o run --output-format csv -- python3 $R/tools/conv_probe.py --case $1 --tile $2 --iters 2 > /dev/null 2>&1 || { echo "pmc b $tag failed"; exit 1; }
  python3 $R/tools/pmc_summary.py $R/gpurun_out/r2s3/probe2/$tag > $R/gpurun_out/r2s3/probe2/$tag.txt 2>&1
  grep -E "patch3|igemm" $R/gpurun_out/r2s3/probe2/$tag.txt | head -2
done
