#!/bin/bash
# Silhouette: its GPU tests, tools/boot_micro.py, then the PMC passes of
# tools/gpu_pmc.sh over tools/sil_micro.py.
mkdir -p gpurun_out/sp
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/sp
timeout -k 10 300 python -u -m pytest tests/test_gpu_edges.py tests/test_gpu_parity.py tests/test_gpu_baseline_shapes.py \
    -k "silhouette or sil" -q -x -p no:cacheprovider -rf --timeout 120 --timeout-method thread > $R/pytest.log 2>&1 || exit $?
timeout -k 10 200 python tools/boot_micro.py > $R/boot_base.log 2>&1 || exit $?
PMC_PROG=tools/sil_micro.py PMC_TAG=sp/pmc bash tools/gpu_pmc.sh || exit $?
