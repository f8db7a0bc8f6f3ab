#!/bin/bash
# Kernel timelines (rocprofv3 --kernel-trace, graphs ON) of the single-graph step and of the
# segmented multi-rank step over a world-1 RCCL process group; gaps by tools/trace_gaps.py.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/trace_one -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 4 > $R/gpurun_out/trace_one.log 2>&1 || { echo "trace one FAILED"; tail -20 $R/gpurun_out/trace_one.log; exit 1; }
python3 $R/tools/trace_gaps.py $R/gpurun_out/trace_one/run_kernel_trace.csv --last 4 > $R/gpurun_out/gaps_one.txt 2>&1; cat $R/gpurun_out/gaps_one.txt
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29633 DBX_FORCE_PG=1 DBX_SEGMENTED_GRAPHS=1
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/trace_seg -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 4 > $R/gpurun_out/trace_seg.log 2>&1 || { echo "trace seg FAILED"; tail -20 $R/gpurun_out/trace_seg.log; exit 1; }
python3 $R/tools/trace_gaps.py $R/gpurun_out/trace_seg/run_kernel_trace.csv --last 4 > $R/gpurun_out/gaps_seg.txt 2>&1; cat $R/gpurun_out/gaps_seg.txt
rm -f $R/gpurun_out/trace_one/run_kernel_trace.csv.gz
