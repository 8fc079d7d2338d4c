#!/bin/bash
# A quick GPU step: -m gpu tests selected by PYTEST_K (skip with PYTEST_K=none),
# smoke, boot_micro (isolated stage times) and the default bench line.  Each
# step under its own time limit; stops at the first failure.  Output:
# gpurun_out/$OUT.
OUT=${OUT:-step}
mkdir -p gpurun_out/$OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/$OUT
if [ "${PYTEST_K:-none}" != "none" ]; then
timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 180 \
    --timeout-method thread -rf -k "$PYTEST_K" > $R/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $R/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.log 2>&1 || exit $?
if [ -z "$NO_MICRO" ]; then
timeout -k 10 240 python tools/boot_micro.py > $R/boot_micro.json 2> $R/boot_micro.err || exit $?
fi
if [ -z "$NO_BENCH" ]; then
timeout -k 10 400 python bench.py --steps ${BSTEPS:-5} --warmup 1 ${BENCH_EXTRA:---no-cpu-baseline} > $R/bench.json 2> $R/bench.err || exit $?
fi
exit 0
