#!/bin/bash
# rocprofv3 kernel stats of one program: KS_PROG (python file), KS_TAG (output name).
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/ks_${KS_TAG:-run}
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R -o run -- \
    python3 $GRAFT_REPO_ROOT/${KS_PROG:-tools/snn_micro.py} > $R.log 2>&1
