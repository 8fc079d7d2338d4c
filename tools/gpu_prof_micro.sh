#!/bin/bash
# Kernel stats of the isolated stage timings (tools/boot_micro.py) under
# rocprofv3 --kernel-trace --stats.  Output: gpurun_out/$OUT.
OUT=${OUT:-profm}
mkdir -p gpurun_out/$OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/$OUT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/stats -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/boot_micro.py > $R/boot_micro.json 2> $R/prof.log || exit $?
exit 0
