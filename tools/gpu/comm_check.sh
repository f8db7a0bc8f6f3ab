#!/bin/bash
# Collective-path checks on one GPU: the direct two-shot kernel (in-process ranks), the framework
# communicator (non-blocking init, captured check, loopback post order of the one-graph step), the
# Composer native_module test (gradient layout), the world-1 RCCL bench with the watchdog / replica
# check and the collective bandwidth tool on every path.
set -o pipefail
O=${1:-gpurun_out/comm_check}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_direct_ar_gpu.py \
  tests/test_comm_gpu.py "tests/test_program_gpu.py::test_composer_trainer_runs_on_native_module" -W always \
  > $O/pytest.log 2>&1; rc=$?; tail -30 $O/pytest.log; [ $rc = 0 ] || exit $rc
grep -c "layout contract" $O/pytest.log || true
DBX_FORCE_PG=1 DBX_ENGINE=segmented_graphs=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29711 bench.py --gpus 1 --steps 15 --warmup 5 > $O/bench_rccl_world1.log 2>&1 \
  || { tail -20 $O/bench_rccl_world1.log; exit 1; }
grep '"metric"' $O/bench_rccl_world1.log | cut -c1-200
DBX_FORCE_PG=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29712 tools/bench_allreduce.py --path all --iters 10 > $O/bench_allreduce_world1.log 2>&1 \
  || { tail -20 $O/bench_allreduce_world1.log; exit 1; }
grep -v '^{' $O/bench_allreduce_world1.log | tail -30
