#!/bin/bash
# Validation of the tree on one GPU: the full GPU suite, smoke, every bench line (headline twice, ZeRO-1,
# presets, the world-1 RCCL one-graph step, two gloo ranks on the device), then the headline kernel profile.
set -o pipefail
O=${1:-gpurun_out/validate}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for p in headline resnet50_imagenet_zero1 resnet50_tiny_imagenet resnet18_cifar10 headline; do
  args="--steps 20 --warmup 5"; [ $p != headline ] && args="$args --preset $p"
  timeout -k 10 300 python bench.py $args > $O/bench_$p.log 2>&1 || { tail -20 $O/bench_$p.log; exit 1; }
  grep '"metric"' $O/bench_$p.log >> $O/bench_lines.txt
  echo "$p: $(grep -o '"value": [0-9.]*' $O/bench_$p.log)"
done
DBX_FORCE_PG=1 DBX_ENGINE=segmented_graphs=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29711 bench.py --gpus 1 --steps 15 --warmup 5 > $O/bench_rccl_world1.log 2>&1 \
  || { tail -20 $O/bench_rccl_world1.log; exit 1; }
grep '"metric"' $O/bench_rccl_world1.log >> $O/bench_lines.txt
echo "headline world-1 RCCL one-graph: $(grep -o '"value": [0-9.]*' $O/bench_rccl_world1.log)"
# two ranks on the one device over gloo (the c10d segmented step, replica checks at world 2)
DBX_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --preset resnet18_cifar10 --steps 10 --warmup 3 \
  > $O/bench_gloo2.log 2>&1 || { tail -20 $O/bench_gloo2.log; exit 1; }
grep '"metric"' $O/bench_gloo2.log >> $O/bench_lines.txt
grep "replicas in sync" $O/bench_gloo2.log
# a multi-rank number measured after a fallback (fresh-rank re-run or c10d rebuild) is not a pass
if grep -q '"comm_fallback": "' $O/bench_lines.txt; then echo "a bench line fell back: $(grep -o '"comm_fallback": "[^"]*"' $O/bench_lines.txt)"; exit 1; fi
bash tools/gpu/profile_headline.sh $O/prof
