#!/bin/bash
# Round-6 A/B of the bench's launch sets: cfg3 (and cfg3job) with
# --boot-batch / --streams variants (AB="nbb,streams,workload ..."), each run
# under its own limit; stops at the first failure.  Output: gpurun_out/$OUT.
OUT=${OUT:-ab6}
R=$GRAFT_REPO_ROOT/gpurun_out/$OUT
mkdir -p $R
export TMPDIR=/tmp
for v in ${AB:-"16,2,cfg3"}; do
  IFS=, read nbb st wl <<< "$v"
  echo "$(date +%T) bench $wl boot-batch $nbb streams $st" >> $R/progress.log
  timeout -k 10 ${BT:-300} python bench.py --workload $wl --steps ${BSTEPS:-5} --warmup 1 --boot-batch $nbb \
      --streams $st ${BENCH_EXTRA:---no-cpu-baseline} > $R/bench_${wl}_b${nbb}_s${st}.json 2> $R/bench_${wl}_b${nbb}_s${st}.err \
      || exit $?
done
exit 0
