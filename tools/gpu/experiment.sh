#!/bin/bash
# One schedule / kernel experiment: GPU tests first, an optional kernel trace under one setting (step
# timeline + per-queue report), then ROUNDS interleaved bench runs of every setting on the presets.
#
#   experiment.sh OUT [-k TEST_FILTER] [-f "TEST_FILES"] [-s TEST_SETTING] [-t SETTING] [-q TRACE_PRESET]
#                     [-p "PRESETS"] [-r ROUNDS] [-m] setting...
#
# A setting is a space-free list of VAR=VALUE joined by '+', or "base" (sweep_env.sh's syntax) -- engine
# switches are DBX_ENGINE=field=v,field=v (engine_config.py); -s sets one for the tests (e.g. a kernel
# switch whose numerics they check). -m runs everything as the world-1 RCCL one-graph multi-rank step
# (the framework communicator's path; segmented_graphs=1 is added to the setting's DBX_ENGINE).
# Examples (the round-5 jobs this replaces; their profile READMEs name them):
#   experiment.sh gpurun_out/ds_fwd -k "side_stream_bit_identical and dsf" -t DBX_ENGINE=ds_fwd_side=1 \
#       -p "headline resnet50_tiny_imagenet" base DBX_ENGINE=ds_fwd_side=0
#   experiment.sh gpurun_out/comm_side -f "tests/test_comm_gpu.py tests/test_multirank_gpu.py" -m \
#       -t DBX_ENGINE=comm_loopback=2 -q resnet50_tiny_imagenet DBX_ENGINE=comm_loopback=2 \
#       DBX_ENGINE=comm_side=0,comm_loopback=2
set -o pipefail
O=$1; shift
FILTER=""; TS=""; MR=""; FILES="tests/test_program_gpu.py"; TRACE=""; TQ="headline"; PRESETS="headline resnet50_tiny_imagenet resnet18_cifar10"; R=2
while getopts "k:f:s:t:q:p:r:m" opt; do
  case $opt in
    k) FILTER=$OPTARG ;; s) TS=${OPTARG//+/ } ;; f) FILES=$OPTARG ;; t) TRACE=$OPTARG ;; q) TQ=$OPTARG ;; p) PRESETS=$OPTARG ;; r) R=$OPTARG ;;
    m) MR=1 ;;
    *) exit 2 ;;
  esac
done
shift $((OPTIND - 1))
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$FILTER" ] || [ "$FILES" != tests/test_program_gpu.py ]; then
  k=(); [ -n "$FILTER" ] && k=(-k "$FILTER")
  env $TS timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread $FILES "${k[@]}" > $O/pytest.log 2>&1
  rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || exit 1
fi
# (the world-1 multi-rank environment is set after the tests: they start their own process groups)
[ -n "$MR" ] && export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29733 \
  DBX_FORCE_PG=1 DBX_ENGINE=segmented_graphs=1
# a setting's VAR=VALUE list as env words; under -m its DBX_ENGINE keeps segmented_graphs=1
envs_of() {
  local s="${1//+/ }" out="" w
  [ "$1" = base ] && s=""
  for w in $s; do
    if [ -n "$DBX_ENGINE" ] && [ "${w%%=*}" = DBX_ENGINE ]; then w="DBX_ENGINE=$DBX_ENGINE,${w#DBX_ENGINE=}"; fi
    out="$out $w"
  done
  echo "$out"
}
if [ -n "$TRACE" ]; then
  envs=$(envs_of "$TRACE")
  a="--steps 6 --warmup 3"; [ $TQ != headline ] && a="$a --preset $TQ"
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o run -- python3 bench.py $a \
    > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
  t=$(find $O/rp -name "*kernel_trace.csv" | head -1)
  python3 tools/step_timeline.py $t --steps 1 --tail 0 --gap-us 300 --top-gaps 4 > $O/timeline.txt 2>&1
  python3 tools/queue_report.py $t --steps 1 > $O/queues.txt 2>&1
  cat $O/timeline.txt $O/queues.txt
fi
[ $# -gt 0 ] || exit 0
for r in $(seq 1 $R); do
  bash tools/gpu/sweep_env.sh $O/r$r "$PRESETS" "$@" || exit 1
done
