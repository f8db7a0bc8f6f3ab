#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r2s3
T="tests/test_program_gpu.py::test_baseline_config_loss_decreases"
for cfg in "DBX_PATCH3=all DBX_STEM_PATCH=1" "DBX_PATCH3=0 DBX_STEM_PATCH=0" "DBX_PATCH3=0 DBX_STEM_PATCH=1" "DBX_PATCH3=all DBX_STEM_PATCH=0" "DBX_FOLD_MAX_RATIO=inf"; do
  env $cfg timeout -k 10 200 python -u -m pytest -q -s --timeout 120 --timeout-method thread -m gpu "$T" -k "sgd" > gpurun_out/r2s3/loss.log 2>&1
  echo "$cfg: $(grep loss50 gpurun_out/r2s3/loss.log | head -1) $(tail -1 gpurun_out/r2s3/loss.log)"
done
