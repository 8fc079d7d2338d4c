#!/bin/bash
# Bench schedules: the default (--streams 3) and each --pipeline NK,NS given as an argument.
mkdir -p gpurun_out/sched
R=gpurun_out/sched
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/default.json 2> $R/default.err || exit $?
for p in "$@"; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --pipeline $p > $R/p$p.json 2> $R/p$p.err || exit $?
done
