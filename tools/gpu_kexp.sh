#!/bin/bash
# kNN micro-benchmark (tools/knn_micro.py, library timers) for several libccg
# variant builds (tools/build_variant.sh): VARIANTS="a b" bash tools/gpu_kexp.sh
mkdir -p gpurun_out/kexp
export TMPDIR=/tmp
for v in ${VARIANTS}; do
  timeout -k 10 300 python3 tools/knn_micro.py --lib tools/variants/libccg_$v.so > gpurun_out/kexp/$v.log 2>&1 || exit $?
done
