#!/bin/bash
# A/B: the GPU tests in $TESTS with the default build, then tools/boot_micro.py
# for the default build and each variant named on the command line.
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/ab
TESTS="${TESTS:-tests/test_gpu_knn_boot.py tests/test_gpu_edges.py tests/test_gpu_baseline_shapes.py}"
timeout -k 10 500 python -u -m pytest $TESTS -q -x -p no:cacheprovider -rf \
    --timeout 120 --timeout-method thread > $R/pytest.log 2>&1 || exit $?
timeout -k 10 200 python tools/boot_micro.py > $R/boot_base.log 2>&1 || exit $?
for v in "$@"; do
  timeout -k 10 200 python tools/boot_micro.py --lib tools/variants/libccg_$v.so > $R/boot_$v.log 2>&1 || exit $?
done
