#!/bin/bash
# Round 4 second call: headline kernel profile (in order and with the default side stream) under the
# current tree, then the multi-rank step benches (world-1 RCCL rehearsal) on the three presets.
set -o pipefail
O=${1:-gpurun_out/r4_s2}
mkdir -p $O
bash tools/gpu/profile_headline.sh $O/prof || exit 1
bash tools/gpu/r4_comm_bench.sh $O/comm
