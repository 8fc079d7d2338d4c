#!/bin/bash
# rocprofv3 kernel statistics of one bench configuration (BENCH_ARGS), each
# step under its own limit.  Output: gpurun_out/$OUT/stats (CSV) + the line.
OUT=${OUT:-prof6}
R=$GRAFT_REPO_ROOT/gpurun_out/$OUT
mkdir -p $R
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/stats -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps ${BSTEPS:-3} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} \
    > $R/prof_bench.json 2> $R/prof.log || exit $?
exit 0
