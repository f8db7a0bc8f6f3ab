#!/bin/bash
# Full validation on one GPU: GPU tests, smoke, bench (headline + presets), phase timing, kernel profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/test_gpu.log 2>&1 || { echo "GPU tests FAILED"; tail -40 gpurun_out/test_gpu.log; exit 1; }
tail -1 gpurun_out/test_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke FAILED"; tail -20 gpurun_out/smoke.log; exit 1; }
echo "smoke ok"
DBX_DIST_BACKEND=gloo timeout -k 10 400 python -m dbx_distributed_pytorch_examples_amd.launch --nproc-per-node 2 tools/dist_gpu_check.py > gpurun_out/dist_check.log 2>&1 || { echo "dist check FAILED"; tail -20 gpurun_out/dist_check.log; exit 1; }
grep "dist_gpu_check" gpurun_out/dist_check.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench FAILED"; tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
for p in resnet50_imagenet_zero1 resnet18_cifar10 resnet50_tiny_imagenet; do
  timeout -k 10 300 python bench.py --preset $p --steps 20 --warmup 5 > gpurun_out/bench_$p.log 2>&1 || { echo "bench $p FAILED"; tail -20 gpurun_out/bench_$p.log; exit 1; }
  echo "$p: $(tail -1 gpurun_out/bench_$p.log | cut -c90-170)"
done
timeout -k 10 300 python bench.py --preset resnet50_imagenet_zero1 --impl torch --steps 10 --warmup 3 > gpurun_out/bench_torch_zero1cfg.log 2>&1 && echo "torch adamw b256: $(tail -1 gpurun_out/bench_torch_zero1cfg.log | cut -c90-170)"
timeout -k 10 300 python bench.py --preset resnet18_cifar10 --impl torch --steps 20 --warmup 5 > gpurun_out/bench_torch_r18.log 2>&1 && echo "torch r18 cifar: $(tail -1 gpurun_out/bench_torch_r18.log | cut -c90-170)"
timeout -k 10 300 python bench.py --preset resnet50_tiny_imagenet --impl torch --steps 20 --warmup 5 > gpurun_out/bench_torch_tiny.log 2>&1 && echo "torch r50 tiny: $(tail -1 gpurun_out/bench_torch_tiny.log | cut -c90-170)"
DBX_PROFILE_PHASES=1 timeout -k 10 300 python tools/phase_times.py > gpurun_out/phases.log 2>&1 && cat gpurun_out/phases.log
cd /tmp && DBX_GRAPHS=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_b1024 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_b1024.log 2>&1; echo "prof rc=$?"
