#!/bin/bash
# A/B a kernel variant build (_C_variant_$1) against the default build inside one box:
# alternating bench runs + the conv tuner sums (fwd/dgrad/wgrad) for each.
set -o pipefail
V=$1
mkdir -p gpurun_out
for r in 1 2; do
  for v in "" "$V"; do
    DBX_EXT_VARIANT=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "variant='$v' $(tail -1 gpurun_out/ab.log | cut -c90-125)"
  done
done
for v in "" "$V"; do
  DBX_EXT_VARIANT=$v timeout -k 10 600 python tools/tune_conv.py --modes fwd,dgrad1,dgrad2,wgrad --out gpurun_out/t_$v.json --report gpurun_out/tune_ab_$v.md > gpurun_out/t.log 2>&1 || { tail -20 gpurun_out/t.log; exit 1; }
done
python - "$V" <<'PY'
import sys
def load(p):
    d={}
    for l in open(p):
        c=[x.strip() for x in l.split('|')]
        if len(c)>8 and c[5] not in ('mode','') and not c[5].startswith('-'):
            d[(c[1],c[2],c[3],c[5])]=(float(c[7]), int(c[4]))
    return d
a=load('gpurun_out/tune_ab_.md'); b=load('gpurun_out/tune_ab_%s.md' % sys.argv[1])
for m in ['fwd','dgrad1','dgrad2','wgrad']:
    ka=[k for k in a if k[3]==m and k in b]
    print(m, round(sum(a[k][0]*a[k][1] for k in ka),3), round(sum(b[k][0]*b[k][1] for k in ka),3))
PY
