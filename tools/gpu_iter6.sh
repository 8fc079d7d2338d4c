#!/bin/bash
# A/B iteration: GPU tests ($TESTS), tools/boot_micro.py for the default build
# and the per-row expansion variant, the co-cluster micro (default vs the
# direct epilogue), and the bench.
mkdir -p gpurun_out/it6
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/it6
TESTS="${TESTS:-tests/test_gpu_knn_boot.py tests/test_gpu_edges.py tests/test_gpu_parity.py tests/test_gpu_baseline_shapes.py}"
timeout -k 10 600 python -u -m pytest $TESTS -q -x -p no:cacheprovider -rf \
    --timeout 120 --timeout-method thread > $R/pytest.log 2>&1 || exit $?
timeout -k 10 200 python tools/boot_micro.py > $R/boot_base.log 2>&1 || exit $?
timeout -k 10 200 python tools/boot_micro.py --lib tools/variants/libccg_expwave0.so > $R/boot_expwave0.log 2>&1 || exit $?
for B in 125 1000; do
  CM_B=$B timeout -k 10 200 python tools/coc_micro.py > $R/coc_base_B$B.log 2>&1 || exit $?
  CM_B=$B timeout -k 10 200 python tools/coc_micro.py --lib tools/variants/libccg_epiold.so > $R/coc_epiold_B$B.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/bench.log 2>&1 || exit $?
