#!/bin/bash
# GPU validation: every -m gpu test (no -x: report all failures), then smoke,
# then a short bench.  Stops at the first crash-like exit (fault/abort/timeout).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 180 --timeout-method thread \
    -rf -k "${PYTEST_K:-not nothing}" > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
src=$?
echo "smoke rc=$src" >> gpurun_out/smoke.log
if [ $src -ne 0 ]; then exit $src; fi
if [ -n "$NO_BENCH" ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 3 --warmup 1 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
brc=$?
echo "bench rc=$brc" >> gpurun_out/bench_quick.err
[ $brc -ne 0 ] && exit $brc
exit $rc
