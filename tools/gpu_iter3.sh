#!/bin/bash
# Iteration check (round 3): the GPU tests named in $TESTS, the silhouette
# micro and a short default bench, each under rocprofv3 kernel stats.  Stops
# at the first failing step.
mkdir -p gpurun_out/it3
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/it3
TESTS="${TESTS:-tests/test_gpu_knn_boot.py tests/test_gpu_edges.py}"
timeout -k 10 500 python -u -m pytest $TESTS -q -x -p no:cacheprovider -rf \
    --timeout 120 --timeout-method thread > $R/pytest.log 2>&1 || exit $?
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/sil -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/sil_micro.py > $R/sil.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/bench -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/bench.log 2>&1 || exit $?
