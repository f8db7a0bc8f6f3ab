#!/bin/bash
# run one test selection (-k EXPR) in each bisect/<commit> worktree and at the repo root
# usage: tools/gpu/bisect_test.sh OUT EXPR [dirs...]
set -o pipefail
O=$1; K=$2; shift 2
mkdir -p $O
for d in "$@" .; do
  n=$(basename $(cd $d && pwd))
  (cd $d && timeout -k 10 300 python -u -m pytest tests/test_program_gpu.py -k "$K" -x -q -s --timeout 200 --timeout-method thread) > $O/$n.log 2>&1
  rc=$?
  echo "$n rc=$rc $(grep -o 'grad-cos.*' $O/$n.log | tr '\n' ' ' | cut -c1-400)"
  [ $rc = 0 ] || [ $rc = 1 ] || exit $rc
done
