#!/bin/bash
# SNN iteration on the GPU: the SNN parity tests, the cfg3 micro-benchmark
# (tools/snn_micro.py), then its kernel trace.  Stops at the first crash-like exit.
mkdir -p gpurun_out/snn
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    -k "${PYTEST_K:-snn}" > gpurun_out/snn/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/snn/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/snn_micro.py > gpurun_out/snn/micro.log 2> gpurun_out/snn/micro.err || exit $?
[ -n "$NO_PROF" ] && exit 0
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/snn/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/snn_micro.py > $GRAFT_REPO_ROOT/gpurun_out/snn/prof.log 2>&1
