#!/bin/bash
# Iteration check (round 3): the GPU tests named in $TESTS, the silhouette
# micro and the default bench (table K 56, then 48), under rocprofv3 kernel
# stats.  Stops at the first failing step.
mkdir -p gpurun_out/it3
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/it3
TESTS="${TESTS:-tests/test_gpu_knn_boot.py tests/test_gpu_edges.py tests/test_gpu_parity.py}"
timeout -k 10 500 python -u -m pytest $TESTS -q -x -p no:cacheprovider -rf \
    --timeout 120 --timeout-method thread > $R/pytest.log 2>&1 || exit $?
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/sil -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/sil_micro.py > $R/sil.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/bench -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/bench.log 2>&1 || exit $?
timeout -k 10 300 python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 1 --table-k 48 \
    > $R/bench48.log 2>&1 || exit $?
for v in 8:3 8:4 8:6; do
  q=${v%%:*}; s=${v##*:}
  timeout -k 10 300 python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 1 --hw-queues $q --streams $s \
      > $R/bench_q${q}_s${s}.log 2>&1 || exit $?
done
cd $GRAFT_REPO_ROOT
for v in base nostore; do
  lib=""; [ $v != base ] && lib="--lib tools/variants/libccg_$v.so"
  CM_B=125 timeout -k 10 200 python tools/coc_micro.py $lib > $R/coc_${v}_B125.log 2>&1 || exit $?
done
