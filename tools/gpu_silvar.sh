#!/bin/bash
# Silhouette kernel stats for the default build and each tools/variants/libccg_<name>.so
# given as arguments: rocprofv3 kernel traces of tools/sil_micro.py.
mkdir -p gpurun_out/silvar
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/silvar
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/base -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/sil_micro.py > $R/base.log 2>&1 || exit $?
for v in "$@"; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$v -o run -- \
      python3 $GRAFT_REPO_ROOT/tools/sil_micro.py --lib $GRAFT_REPO_ROOT/tools/variants/libccg_$v.so > $R/$v.log 2>&1 || exit $?
done
