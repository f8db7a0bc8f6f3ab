#!/bin/bash
# PMC passes (kernel-trace only) for the forward 1x1 / 3x3 convs with prologue + stats epilogue.
set -o pipefail
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for shape in "1024 64 256 56 1 fwdps" "1024 256 256 14 3 fwdps"; do
  tag=$(echo $shape | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc2/${tag}_a -o run --output-format csv -- python3 $R/tools/wgrad_one.py $shape > $R/gpurun_out/pmc2/${tag}_a.log 2>&1 || { echo "pmc $tag a failed"; tail -5 $R/gpurun_out/pmc2/${tag}_a.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS -d $R/gpurun_out/pmc2/${tag}_b -o run --output-format csv -- python3 $R/tools/wgrad_one.py $shape > $R/gpurun_out/pmc2/${tag}_b.log 2>&1 || { echo "pmc $tag b failed"; tail -5 $R/gpurun_out/pmc2/${tag}_b.log; exit 1; }
  echo "pmc $tag ok"
done
