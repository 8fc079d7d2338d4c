#!/bin/bash
# Round-5 profiling step: isolated per-stage times (tools/boot_micro.py, both
# SNN passes), the default bench under rocprofv3 --kernel-trace --stats, and
# PMC passes over boot_micro (one counter group per run).  Each step has its
# own time limit; stops at the first failure.  Output: gpurun_out/$OUT.
OUT=${OUT:-prof5}
mkdir -p gpurun_out/$OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/$OUT
if [ -z "$NO_MICRO" ]; then
BM_SNN=classes timeout -k 10 240 python tools/boot_micro.py > $R/boot_micro_classes.json 2> $R/boot_micro.err || exit $?
BM_SNN=rows timeout -k 10 240 python tools/boot_micro.py > $R/boot_micro_rows.json 2>> $R/boot_micro.err || exit $?
fi
cd /tmp
if [ -z "$NO_STATS" ]; then
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/stats -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_EXTRA:-} > $R/prof_bench.json 2> $R/prof.log || exit $?
fi
IFS=';' read -ra GRP <<< "${PMC_GROUPS:-}"
i=0
for g in "${GRP[@]}"; do
  BM_BOOTS=4 timeout -s KILL 150 rocprofv3 --pmc $g --output-format csv -d $R/pmc/pass_$i -o run -- \
      python3 $GRAFT_REPO_ROOT/tools/boot_micro.py > $R/pmc_$i.log 2>&1 || exit $?
  i=$((i+1))
done
exit 0
