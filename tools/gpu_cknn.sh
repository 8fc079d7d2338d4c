#!/bin/bash
# Consensus kNN: its GPU tests (edges, scale), then tools/cknn_micro.py.
mkdir -p gpurun_out/ck
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/ck
timeout -k 10 600 python -u -m pytest tests/test_gpu_edges.py tests/test_gpu_scale.py tests/test_gpu_parity.py -q -x \
    -p no:cacheprovider -rf --timeout 300 --timeout-method thread > $R/pytest.log 2>&1 || exit $?
timeout -k 10 200 python tools/cknn_micro.py > $R/cknn.json 2> $R/cknn.err || exit $?
