#!/bin/bash
# kNN micro-benchmark: the product screen and its timing/tuning variants.
# KNN_VARIANTS: space-separated EXP[:QF] pairs (CCG_KNN_EXP, CCG_KNN_QF).
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/micro.log
for v in ${KNN_VARIANTS:-0 1 2 3}; do
  e=${v%%:*}; q=""; [ "$v" != "$e" ] && q=${v#*:}
  CCG_KNN_EXP=$e CCG_KNN_QF=$q timeout -k 10 300 python tools/knn_micro.py >> gpurun_out/micro.log 2>>gpurun_out/micro.err || exit $?
done
