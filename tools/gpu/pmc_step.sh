#!/bin/bash
# Per-kernel PMC counters over one eager ResNet-50 b1024 training step (wgrad side stream off so
# dispatches do not overlap). Two passes, kernel-trace only (no sys/runtime trace with --pmc).
# Output: gpurun_out/pmc_step/{a,b}/run_counter_collection.csv; summary by tools/pmc_summary.py
set -o pipefail
O=${2:-gpurun_out/pmc_step}
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B=${1:-1024}
cd /tmp
export DBX_ENGINE=graphs=0,overlap_wgrad=0
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $R/$O/a -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --batch $B > $R/$O/a.log 2>&1 || { echo "pmc a failed"; tail -5 $R/$O/a.log; exit 1; }
echo "pass a ok"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum -d $R/$O/b -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --batch $B > $R/$O/b.log 2>&1 || { echo "pmc b failed"; tail -5 $R/$O/b.log; exit 1; }
echo "pass b ok"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/$O/c -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --batch $B > $R/$O/c.log 2>&1 || { echo "pmc c failed"; tail -5 $R/$O/c.log; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/$O/d -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --batch $B > $R/$O/d.log 2>&1 || { echo "pmc d failed"; tail -5 $R/$O/d.log; exit 1; }
echo "passes c, d ok"
python3 $R/tools/pmc_summary.py $R/$O > $R/$O/summary.txt 2>&1 || echo "summary failed (raw CSVs kept)"
head -60 $R/$O/summary.txt
