#!/bin/bash
# rocprofv3 kernel stats of the default bench command (isolated streams=1 and
# default), written to gpurun_out/prof_<tag>/.  Usage: TAG=r02a bash tools/gpu_prof_bench.sh
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-prof}
R=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_${T}_default -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 3 ${BENCH_ARGS} > $R/prof_${T}_default.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_${T}_streams1 -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --streams 1 --boots-per-gpu 32 --steps 2 ${BENCH_ARGS} \
    > $R/prof_${T}_streams1.log 2>&1 || exit $?
exit 0
