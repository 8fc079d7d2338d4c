#!/bin/bash
# Quick GPU iteration: selected parity tests (PYTEST_K) then a short bench.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    -k "${PYTEST_K:-.}" > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_quick.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench_quick.log 2> gpurun_out/bench_quick.err
