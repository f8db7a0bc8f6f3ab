#!/bin/bash
# Round 4: small-step defaults (4 statistics shards, consumer-side forward finalize, block-cooperative
# backward finalize in the BN-backward apply passes): bit-exactness, then the three configs against
# the previous defaults.
set -o pipefail
O=${1:-gpurun_out/r4_s7}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_bn_fin_gpu.py tests/test_comm_gpu.py -x -q --timeout 200 \
  --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
bash tools/gpu/sweep_env.sh $O "resnet18_cifar10 resnet50_tiny_imagenet" base DBX_COEFF_IN=0 \
  DBX_NSHARD=32+DBX_FIN_IN=0+DBX_COEFF_IN=0 base
bash tools/gpu/sweep_env.sh $O "headline" base DBX_NSHARD=4+DBX_COEFF_IN=1 base
