#!/bin/bash
# Time libccg variants (tools/variants/libccg_<name>.so) with a micro-benchmark.
# VARIANTS="a b c" PROG=tools/knn_micro.py bash tools/gpu_variants.sh
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/variants.log
for v in ${VARIANTS}; do
  for rep in 1 2; do
    echo -n "$v " >> gpurun_out/variants.log
    timeout -k 10 300 python ${PROG:-tools/knn_micro.py} --lib tools/variants/libccg_$v.so >> gpurun_out/variants.log 2>>gpurun_out/variants.err || exit $?
  done
done
