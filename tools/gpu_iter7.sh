#!/bin/bash
# Round-3 iteration: GPU tests ($TESTS), tools/boot_micro.py (default vs the
# per-row expansion), the co-cluster micro (default vs the direct epilogue;
# B = 125 with bench-like C ~ 37, and B = 1000), the FETCH/WRITE PMC passes
# of the co-cluster micro (traffic), and the bench.
mkdir -p gpurun_out/it7
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/it7
TESTS="${TESTS:-tests/test_gpu_knn_boot.py tests/test_gpu_edges.py tests/test_gpu_parity.py tests/test_gpu_baseline_shapes.py}"
timeout -k 10 600 python -u -m pytest $TESTS -q -x -p no:cacheprovider -rf \
    --timeout 120 --timeout-method thread > $R/pytest.log 2>&1 || exit $?
timeout -k 10 200 python tools/boot_micro.py > $R/boot_base.log 2>&1 || exit $?
timeout -k 10 200 python tools/boot_micro.py --lib tools/variants/libccg_expwave0.so > $R/boot_expwave0.log 2>&1 || exit $?
for v in base epiold; do
  lib=""; [ $v != base ] && lib="--lib tools/variants/libccg_$v.so"
  CM_B=125 CM_CLO=30 CM_CHI=44 timeout -k 10 200 python tools/coc_micro.py $lib > $R/coc_${v}_B125.log 2>&1 || exit $?
  CM_B=1000 timeout -k 10 200 python tools/coc_micro.py $lib > $R/coc_${v}_B1000.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/bench.log 2>&1 || exit $?
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  CM_B=125 CM_CLO=30 CM_CHI=44 timeout -k 10 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $R/pmc/$c -o run -- \
      python3 $GRAFT_REPO_ROOT/tools/coc_micro.py > $R/pmc_$c.log 2>&1 || exit $?
done
