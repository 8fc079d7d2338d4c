#!/bin/bash
# rocprofv3 kernel stats of a micro-benchmark for several libccg variant builds.
# VARIANTS="base x" PROG=tools/knn_micro.py bash tools/gpu_kvar.sh -> gpurun_out/ks_<variant>/
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp
for v in ${VARIANTS}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/ks_$v -o run -- \
      python3 $GRAFT_REPO_ROOT/${PROG:-tools/knn_micro.py} --lib $GRAFT_REPO_ROOT/tools/variants/libccg_$v.so \
      > $R/ks_$v.log 2>&1 || exit $?
done
