#!/bin/bash
# Round-5 measurement step: smoke, isolated stage times (tools/boot_micro.py),
# the default bench line (HIP-graph launch), the same bench with eager
# launches, and the default bench under rocprofv3 --kernel-trace --stats.
# Each step has its own time limit; stops at the first failure.
# Output: gpurun_out/$OUT.
OUT=${OUT:-bench5}
mkdir -p gpurun_out/$OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/$OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.log 2>&1 || exit $?
timeout -k 10 240 python tools/boot_micro.py > $R/boot_micro.json 2> $R/boot_micro.err || exit $?
timeout -k 10 400 python bench.py --steps ${BSTEPS:-5} --warmup 1 ${BENCH_EXTRA:-} > $R/bench.json 2> $R/bench.err || exit $?
if [ -z "$NO_EAGER" ]; then
timeout -k 10 400 python bench.py --steps ${BSTEPS:-5} --warmup 1 --launch eager --no-cpu-baseline > $R/bench_eager.json 2> $R/bench_eager.err || exit $?
fi
if [ -z "$NO_STATS" ]; then
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/stats -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/prof_bench.json 2> $R/prof.log || exit $?
fi
exit 0
