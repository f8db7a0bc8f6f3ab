#!/bin/bash
# PMC counters of single 3x3 conv kernels (tools/conv_probe.py), one pass per counter group.
set -o pipefail
mkdir -p gpurun_out/r2s3/probe
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for c in "fwd3x3_64 128,64,1" "fwd3x3_64 128,64,0" "dgrad3x3_64 256,64,2" "dgrad3x3_64 256,64,0" "fwd3x3_128 128,128,1" "dgrad3x3_128 128,128,2" "fwd3x3_256 128,256,0" "dgrad3x3_256 128,128,2"; do
  set -- $c
  tag=${1}_${2//,/x}
  timeout -k 10 60 python3 $R/tools/conv_probe.py --case $1 --tile $2 | tee -a $R/gpurun_out/r2s3/probe/times.txt
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $R/gpurun_out/r2s3/probe/$tag/a -o run --output-format csv -- python3 $R/tools/conv_probe.py --case $1 --tile $2 --iters 2 > /dev/null 2>&1 || { echo "pmc a $tag failed"; exit 1; }
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR -d $R/gpurun_out/r2s3/probe/$tag/b -o run --output-format csv -- python3 $R/tools/conv_probe.py --case $1 --tile $2 --iters 2 > /dev/null 2>&1 || { echo "pmc b $tag failed"; exit 1; }
  python3 $R/tools/pmc_summary.py $R/gpurun_out/r2s3/probe/$tag > $R/gpurun_out/r2s3/probe/$tag.txt 2>&1
  grep igemm $R/gpurun_out/r2s3/probe/$tag.txt | head -2
done
