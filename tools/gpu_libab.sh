#!/bin/bash
# A/B of prebuilt libccg variants on the kNN micro-benchmark: LIBS = space-separated
# paths under gpurun_out/libab/ (copied into the package before each run).
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/libab.log
cp consensusclustr_amd/libccg.so /tmp/libccg_orig.so
for l in $LIBS; do
  cp "$l" consensusclustr_amd/libccg.so
  echo "== $l" >> gpurun_out/libab.log
  timeout -k 10 300 python tools/${AB_PROG:-knn_micro.py} >> gpurun_out/libab.log 2>>gpurun_out/libab.err || { cp /tmp/libccg_orig.so consensusclustr_amd/libccg.so; exit 1; }
done
cp /tmp/libccg_orig.so consensusclustr_amd/libccg.so
