#!/bin/bash
# PMC counters for single conv kernels (each counter group in its own run; kernel-trace only)
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
i=0
for shape in "1024 256 256 14 3 wgrad" "1024 256 1024 14 1 wgrad" "1024 256 256 14 3 fwd"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS -d $R/gpurun_out/pmc/a$i -o run --output-format csv -- python3 $R/tools/wgrad_one.py $shape > $R/gpurun_out/pmc/a$i.log 2>&1 || { echo "pmc a$i failed"; tail -5 $R/gpurun_out/pmc/a$i.log; exit 1; }
  timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD TA_BUSY_avr -d $R/gpurun_out/pmc/b$i -o run --output-format csv -- python3 $R/tools/wgrad_one.py $shape > $R/gpurun_out/pmc/b$i.log 2>&1 || { echo "pmc b$i failed"; tail -5 $R/gpurun_out/pmc/b$i.log; exit 1; }
done
echo pmc done
