#!/bin/bash
# SNN class-kernel grid A/B: the SNN GPU tests with the default build, then
# tools/boot_micro.py for the default build and each SNN_GRID variant.
mkdir -p gpurun_out/sg
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/sg
timeout -k 10 300 python -u -m pytest tests/test_gpu_edges.py tests/test_gpu_parity.py -k "snn" -q -x -p no:cacheprovider \
    -rf --timeout 120 --timeout-method thread > $R/pytest.log 2>&1 || exit $?
timeout -k 10 200 python tools/boot_micro.py > $R/boot_base.log 2>&1 || exit $?
for v in "$@"; do
  timeout -k 10 200 python tools/boot_micro.py --lib tools/variants/libccg_$v.so > $R/boot_$v.log 2>&1 || exit $?
done
