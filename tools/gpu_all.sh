#!/bin/bash
# Parity tests -> bench -> rocprofv3 kernel trace; stops at the first crash-like exit.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2> gpurun_out/bench.err || exit $?
if [ -n "$NO_PROF" ]; then exit $rc; fi
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --boots-per-gpu 16 --steps 2 --warmup 1 --no-cpu-baseline \
    > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1 || exit $?
exit $rc
