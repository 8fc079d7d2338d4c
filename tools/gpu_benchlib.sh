#!/bin/bash
# Default bench with each tools/variants/libccg_<name>.so swapped in for the
# package library (on the GPU box's scratch copy of the tree only).
mkdir -p gpurun_out/benchlib
R=gpurun_out/benchlib
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/base.json 2> $R/base.err || exit $?
cp consensusclustr_amd/libccg.so /tmp/libccg_base.so
for v in "$@"; do
  cp tools/variants/libccg_$v.so consensusclustr_amd/libccg.so
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $R/$v.json 2> $R/$v.err || exit $?
done
cp /tmp/libccg_base.so consensusclustr_amd/libccg.so
