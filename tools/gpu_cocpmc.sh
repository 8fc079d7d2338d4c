#!/bin/bash
# Co-cluster at the bench shape (N=100k, B=125): tools/coc_micro.py for the
# default build and the no-store variant, then the PMC passes of
# tools/gpu_pmc.sh over tools/coc_micro.py.
mkdir -p gpurun_out/cp
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/cp
timeout -k 10 200 python tools/coc_micro.py > $R/coc_base.log 2>&1 || exit $?
timeout -k 10 200 python tools/coc_micro.py --lib tools/variants/libccg_nostore.so > $R/coc_nostore.log 2>&1 || exit $?
PMC_PROG=tools/coc_micro.py PMC_TAG=cp/pmc bash tools/gpu_pmc.sh || exit $?
