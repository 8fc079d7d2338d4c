#!/bin/bash
# Kernel trace (--stats) of a short bench run; summary -> gpurun_out/ktrace/
mkdir -p gpurun_out/ktrace
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ktrace -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --boots-per-gpu ${KT_BOOTS:-16} --steps 2 --warmup 1 --no-cpu-baseline \
    > $GRAFT_REPO_ROOT/gpurun_out/ktrace/bench.log 2>&1
