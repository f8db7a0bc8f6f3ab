#!/bin/bash
# Round-2 session-5 final revalidation (frozen-backbone graphs, MDS compression): GPU tests, smoke, presets, RCCL world-1 rehearsal of the
# multi-rank path, headline bench, rocprofv3 kernel stats.
set -o pipefail
mkdir -p gpurun_out/r2s5final
export TMPDIR=/tmp
O=gpurun_out/r2s5final
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/test_gpu.log 2>&1 || { echo "GPU tests FAILED"; tail -40 $O/test_gpu.log; exit 1; }
tail -1 $O/test_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke FAILED"; tail -20 $O/smoke.log; exit 1; }
echo "smoke ok"
export DBX_FORCE_PG=1
L="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
DBX_SEGMENTED_GRAPHS=1 timeout -k 10 300 $L --master-port 29614 tools/dist_gpu_check.py > $O/rccl_check6.log 2>&1 || { echo "rccl check FAILED"; tail -30 $O/rccl_check6.log; exit 1; }
grep dist_gpu_check $O/rccl_check6.log
DBX_SEGMENTED_GRAPHS=1 timeout -k 10 300 $L --master-port 29615 bench.py --gpus 1 --steps 20 --warmup 5 > $O/rccl_bench_seg6.log 2>&1 || { echo "seg6 bench FAILED"; tail -30 $O/rccl_bench_seg6.log; exit 1; }
echo "segmented+RCCL world 1: $(tail -1 $O/rccl_bench_seg6.log | cut -c80-140)"
unset DBX_FORCE_PG
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/bench_default.log 2>&1 || { echo "bench FAILED"; tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
for p in resnet50_imagenet_zero1 resnet18_cifar10 resnet50_tiny_imagenet; do
  timeout -k 10 300 python bench.py --preset $p --steps 20 --warmup 5 > $O/bench_$p.log 2>&1 || { echo "bench $p FAILED"; tail -20 $O/bench_$p.log; exit 1; }
  echo "$p: $(tail -1 $O/bench_$p.log | cut -c80-140)"
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_b1024 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/$O/prof_b1024.log 2>&1; echo "prof rc=$?"
