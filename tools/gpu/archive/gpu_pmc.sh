#!/bin/bash
# PMC counters of single conv kernels (each counter group in its own run; kernel-trace only, no
# sys/runtime trace). Output: gpurun_out/pmc/<tag>_{a,b}/run_counter_collection.csv
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for shape in "1024 256 256 14 3 fwd" "1024 256 256 14 3 dgrad" "1024 256 256 14 3 wgrad" "1024 64 64 56 3 fwd" "1024 256 1024 14 1 fwd"; do
  tag=$(echo $shape | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc/${tag}_a -o run --output-format csv -- python3 $R/tools/wgrad_one.py $shape > $R/gpurun_out/pmc/${tag}_a.log 2>&1 || { echo "pmc $tag a failed"; tail -5 $R/gpurun_out/pmc/${tag}_a.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU TA_BUSY_avr -d $R/gpurun_out/pmc/${tag}_b -o run --output-format csv -- python3 $R/tools/wgrad_one.py $shape > $R/gpurun_out/pmc/${tag}_b.log 2>&1 || { echo "pmc $tag b failed"; tail -5 $R/gpurun_out/pmc/${tag}_b.log; exit 1; }
  echo "pmc $tag ok"
done
echo pmc done
