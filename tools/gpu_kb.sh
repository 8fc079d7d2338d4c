#!/bin/bash
# Distinct-cell kNN iteration: its tests and the other kNN/pipeline tests,
# knn_micro in both modes, a short bench.  Stops at the first crash-like exit.
mkdir -p gpurun_out/kb
R=gpurun_out/kb
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -x \
    -k "${PYTEST_K:-knn or boot or baseline or pipeline or consensus or smoke}" > $R/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $R/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/knn_micro.py > $R/micro_boot.log 2>&1 || exit $?
KM_MODE=rows timeout -k 10 200 python tools/knn_micro.py > $R/micro_rows.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/bench.json 2> $R/bench.err || exit $?
