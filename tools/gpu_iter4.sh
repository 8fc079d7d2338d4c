#!/bin/bash
# Iteration check: GPU tests ($TESTS), the silhouette micro (screened widths,
# the fp64-MFMA widths, the no-fallback timing variant) and the default bench
# at several (hardware queues, streams).  Stops at the first failing step.
mkdir -p gpurun_out/it4
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/it4
TESTS="${TESTS:-tests/test_gpu_knn_boot.py tests/test_gpu_edges.py tests/test_gpu_parity.py}"
timeout -k 10 500 python -u -m pytest $TESTS -q -x -p no:cacheprovider -rf \
    --timeout 120 --timeout-method thread > $R/pytest.log 2>&1 || exit $?
timeout -k 10 200 python tools/sil_micro.py > $R/sil_scr.log 2>&1 || exit $?
CCG_SIL_WIDTH=mfma64 timeout -k 10 200 python tools/sil_micro.py > $R/sil_f64.log 2>&1 || exit $?
timeout -k 10 200 python tools/sil_micro.py --lib tools/variants/libccg_nofb.so > $R/sil_nofb.log 2>&1 || exit $?
for v in 0:3 8:4 8:6 12:8; do
  q=${v%%:*}; s=${v##*:}
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --hw-queues $q --streams $s \
      > $R/bench_q${q}_s${s}.log 2>&1 || exit $?
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/bench -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/bench_prof.log 2>&1 || exit $?
