#!/bin/bash
# Bench (N=1) then a rocprofv3 kernel-trace of a shorter run of the same workload.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2> gpurun_out/bench.err || exit $?
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --boots-per-gpu 16 --steps 2 --warmup 1 --no-cpu-baseline \
    > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
