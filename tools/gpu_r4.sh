#!/bin/bash
# Round-4 GPU step: selected -m gpu tests (PYTEST_K / PYTEST_FILES), then an
# optional short bench.  Stops at the first crash-like exit.
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/r4
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -v -p no:cacheprovider --timeout 180 \
    --timeout-method thread -rf -k "${PYTEST_K:-not nothing}" > $R/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $R/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "$BENCH_ARGS" ]; then
  timeout -k 10 600 python bench.py $BENCH_ARGS > $R/bench.json 2> $R/bench.err
  brc=$?; echo "bench rc=$brc" >> $R/bench.err
  [ $brc -ne 0 ] && exit $brc
fi
exit $rc
