#!/bin/bash
# kNN screen variants: tools/knn_micro.py with the default build and each
# tools/variants/libccg_<name>.so given as an argument (one process each).
mkdir -p gpurun_out/kvar
R=gpurun_out/kvar
timeout -k 10 200 python tools/knn_micro.py > $R/base.log 2>&1 || exit $?
for v in "$@"; do
  timeout -k 10 200 python tools/knn_micro.py --lib tools/variants/libccg_$v.so > $R/$v.log 2>&1 || exit $?
done
