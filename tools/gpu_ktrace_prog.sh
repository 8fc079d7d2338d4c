#!/bin/bash
# Kernel trace (--stats) of a tools/ micro-benchmark: KT_PROG (default snn_micro.py)
mkdir -p gpurun_out/ktp
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ktp -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/${KT_PROG:-snn_micro.py} > $GRAFT_REPO_ROOT/gpurun_out/ktp/run.log 2>&1
