#!/bin/bash
# Bench at each --streams value given as an argument.
mkdir -p gpurun_out/streams
for s in "$@"; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --streams $s > gpurun_out/streams/s$s.json 2> gpurun_out/streams/s$s.err || exit $?
done
