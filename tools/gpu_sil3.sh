#!/bin/bash
# Silhouette check: the silhouette GPU tests, then the silhouette micro under
# rocprofv3 kernel stats.  Stops at the first failing step.
mkdir -p gpurun_out/sil3
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/sil3
timeout -k 10 400 python -u -m pytest tests/test_gpu_edges.py tests/test_gpu_parity.py -k "silhouette" -q -x -p no:cacheprovider -rf \
    --timeout 120 --timeout-method thread > $R/pytest.log 2>&1 || exit $?
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/sil -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/sil_micro.py > $R/sil.log 2>&1 || exit $?
