#!/bin/bash
# kNN iteration on the GPU: the kNN parity tests, the cfg3 micro-benchmark
# (synthetic NB PCs, then a Gaussian mixture), then a short bench.
# Stops at the first crash-like exit.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    -k "${PYTEST_K:-knn}" > gpurun_out/pytest_knn.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_knn.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/knn_micro.py > gpurun_out/knn_micro.log 2> gpurun_out/knn_micro.err || exit $?
KM_DATA=gauss timeout -k 10 300 python tools/knn_micro.py >> gpurun_out/knn_micro.log 2>> gpurun_out/knn_micro.err || exit $?
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
