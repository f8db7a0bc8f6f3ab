#!/bin/bash
# one bench run per environment setting (interleaved per preset):  sweep_env.sh OUT "presets" setting...
# a setting is a space-free list of VAR=VALUE joined by '+', or "base"; a DBX_ENGINE=... of the setting is
# appended to an exported DBX_ENGINE (experiment.sh -m exports segmented_graphs=1)
set -o pipefail
envs_of() {
  local s="${1//+/ }" out="" w
  [ "$1" = base ] && s=""
  for w in $s; do
    if [ -n "$DBX_ENGINE" ] && [ "${w%%=*}" = DBX_ENGINE ]; then w="DBX_ENGINE=$DBX_ENGINE,${w#DBX_ENGINE=}"; fi
    out="$out $w"
  done
  echo "$out"
}
O=$1; PRESETS=$2; shift 2
mkdir -p $O
for p in $PRESETS; do
  for st in "$@"; do
    envs=$(envs_of "$st")
    args="--steps 30 --warmup 10"; [ $p = headline ] && args="--steps 15 --warmup 5" || args="$args --preset $p"
    f=$O/${p}_$(echo "$st" | tr "=+/," "____").log
    env $envs timeout -k 10 300 python bench.py $args > $f 2>&1 || { tail -20 $f; exit 1; }
    echo "$p $st: $(grep -o '"value": [0-9.]*' $f)"
  done
done
