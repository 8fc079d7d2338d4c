#!/bin/bash
# One GPU round step: selected -m gpu tests (PYTEST_FILES, or "none"), smoke
# (SMOKE=1), then bench workloads (WORKLOADS, BSTEPS, BENCH_EXTRA), each step
# under its own time limit; stops at the first failure.  Output: gpurun_out/$OUT.
OUT=${OUT:-r5}
mkdir -p gpurun_out/$OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/$OUT
rc=0
if [ "${PYTEST_FILES:-tests}" != "none" ]; then
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -v -p no:cacheprovider --timeout 180 \
    --timeout-method thread -rf -k "${PYTEST_K:-not nothing}" > $R/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $R/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ -n "$SMOKE" ]; then
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.log 2>&1
src=$?; echo "smoke rc=$src" >> $R/smoke.log
[ $src -ne 0 ] && exit $src
fi
for w in ${WORKLOADS:-}; do
  timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py --workload $w --steps ${BSTEPS:-3} --warmup 1 \
      ${BENCH_EXTRA:---no-cpu-baseline} > $R/bench_$w.json 2> $R/bench_$w.err
  brc=$?; echo "bench rc=$brc" >> $R/bench_$w.err
  [ $brc -ne 0 ] && exit $brc
done
exit $rc
