#!/bin/bash
# Silhouette row vs distinct-cell path (kernel stats) and the default bench's
# kernel stats.
mkdir -p gpurun_out/silprof
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/silprof
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/sil -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/sil_micro.py > $R/sil.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/bench -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 5 --warmup 2 > $R/bench.log 2>&1 || exit $?
