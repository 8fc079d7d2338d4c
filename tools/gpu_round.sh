#!/bin/bash
# One GPU round step: selected -m gpu tests (PYTEST_FILES, or "none"), then bench workloads
# (WORKLOADS, BSTEPS, BENCH_EXTRA), each
# step under its own time limit; stops at the first failure.
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/r4
rc=0
if [ "${PYTEST_FILES:-tests}" != "none" ]; then
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -v -p no:cacheprovider --timeout 180 \
    --timeout-method thread -rf -k "${PYTEST_K:-not nothing}" > $R/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $R/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
for w in ${WORKLOADS:-}; do
  timeout -k 10 400 python bench.py --workload $w --steps ${BSTEPS:-3} --warmup 1 ${BENCH_EXTRA:---no-cpu-baseline} \
      > $R/bench_$w.json 2> $R/bench_$w.err
  brc=$?; echo "bench rc=$brc" >> $R/bench_$w.err
  [ $brc -ne 0 ] && exit $brc
done
exit $rc
