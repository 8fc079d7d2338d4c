#!/bin/bash
# A/B micros only: tools/coc_micro.py (B = 125 at the default and the
# bench-like label counts, B = 1000) for the default build and the co-cluster
# variants in $COC, tools/boot_micro.py for the default build and the
# variants in $BOOT.
mkdir -p gpurun_out/ab2
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/ab2
for v in base $COC; do
  L=""; [ $v != base ] && L="--lib tools/variants/libccg_$v.so"
  timeout -k 10 200 python tools/coc_micro.py $L > $R/coc_${v}_B125.log 2>&1 || exit $?
  CM_CLO=30 CM_CHI=44 timeout -k 10 200 python tools/coc_micro.py $L > $R/coc_${v}_B125c37.log 2>&1 || exit $?
  CM_B=1000 timeout -k 10 200 python tools/coc_micro.py $L > $R/coc_${v}_B1000.log 2>&1 || exit $?
done
for v in base $BOOT; do
  L=""; [ $v != base ] && L="--lib tools/variants/libccg_$v.so"
  BM_BOOTS=16 timeout -k 10 200 python tools/boot_micro.py $L > $R/boot_$v.log 2>&1 || exit $?
done
