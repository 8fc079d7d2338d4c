#!/bin/bash
# A/B iteration: GPU tests ($TESTS), tools/boot_micro.py (one-stream bootstrap
# chain per stage) for the default build and each variant, the co-cluster
# micro for the default and the direct-epilogue variant, and the bench.
mkdir -p gpurun_out/it5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/it5
TESTS="${TESTS:-tests/test_gpu_knn_boot.py tests/test_gpu_edges.py tests/test_gpu_parity.py}"
timeout -k 10 500 python -u -m pytest $TESTS -q -x -p no:cacheprovider -rf \
    --timeout 120 --timeout-method thread > $R/pytest.log 2>&1 || exit $?
timeout -k 10 200 python tools/boot_micro.py > $R/boot_base.log 2>&1 || exit $?
CCG_SIL_WIDTH=mfma64 timeout -k 10 200 python tools/boot_micro.py > $R/boot_silf64.log 2>&1 || exit $?
for v in expold rsfix sumrows; do
  timeout -k 10 200 python tools/boot_micro.py --lib tools/variants/libccg_$v.so > $R/boot_$v.log 2>&1 || exit $?
done
for B in 125 1000; do
  CM_B=$B timeout -k 10 200 python tools/coc_micro.py > $R/coc_base_B$B.log 2>&1 || exit $?
  CM_B=$B timeout -k 10 200 python tools/coc_micro.py --lib tools/variants/libccg_epiold.so > $R/coc_epiold_B$B.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/bench.log 2>&1 || exit $?
CCG_SIL_WIDTH=mfma64 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/bench_silf64.log 2>&1 || exit $?
