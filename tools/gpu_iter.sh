#!/bin/bash
# Iteration check: the GPU tests named in $TESTS (default: the edge, kNN-boot
# and SNN tests), then the silhouette micro and the default bench under
# rocprofv3 kernel stats.  Stops at the first failing step.
mkdir -p gpurun_out/iter
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/iter
TESTS="${TESTS:-tests/test_gpu_edges.py tests/test_gpu_knn_boot.py tests/test_gpu_parity.py}"
timeout -k 10 600 python -u -m pytest $TESTS -q -x -p no:cacheprovider -rf --timeout 180 --timeout-method thread \
    > $R/pytest.log 2>&1 || exit $?
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/sil -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/sil_micro.py > $R/sil.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/bench -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 5 --warmup 2 > $R/bench.log 2>&1 || exit $?
