#!/bin/bash
# native RCCL communicator tests, then the per-op roofline table of the headline step
set -o pipefail
O=${1:-gpurun_out/comm_bd}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_comm_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_comm.log 2>&1
rc=$?; tail -8 $O/pytest_comm.log; [ $rc = 0 ] || exit $rc
BATCH=1024 timeout -k 10 300 python tools/op_breakdown.py --steps 2 --top 70 > $O/op_breakdown.txt 2>&1 || { tail -20 $O/op_breakdown.txt; exit 1; }
head -100 $O/op_breakdown.txt
