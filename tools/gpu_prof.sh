#!/bin/bash
# Kernel trace of a short bench + PMC passes over the kNN micro-benchmark.
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --boots-per-gpu 16 --steps 2 --warmup 1 --no-cpu-baseline \
    > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && bash tools/gpu_pmc.sh
