#!/bin/bash
# Round 4: consumer-side BN finalizes -- the backward coefficients computed by the BN-backward apply
# passes (DBX_COEFF_IN), the forward ones by the consuming conv's prologue (DBX_FIN_IN), with fewer
# statistics shards (DBX_NSHARD) so each consumer reads less: bit-exactness, then all three configs.
set -o pipefail
O=${1:-gpurun_out/r4_s6}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_bn_fin_gpu.py -x -q --timeout 200 --timeout-method thread \
  > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
bash tools/gpu/sweep_env.sh $O "resnet18_cifar10 resnet50_tiny_imagenet headline" base DBX_COEFF_IN=1 \
  DBX_NSHARD=4+DBX_FIN_IN=1 DBX_NSHARD=4+DBX_FIN_IN=1+DBX_COEFF_IN=1 DBX_NSHARD=2+DBX_FIN_IN=1+DBX_COEFF_IN=1 \
  DBX_NSHARD=1+DBX_FIN_IN=1+DBX_COEFF_IN=1 base
