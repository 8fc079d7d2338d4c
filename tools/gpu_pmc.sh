#!/bin/bash
# rocprofv3 --pmc passes of "python3 $PMC_CMD", one counter group per run
# (groups separated by ';'), into gpurun_out/pmc/pass_<i>; each pass under its
# own kill timeout; stops at the first failure.  Output directory
# gpurun_out/$PMC_OUT (default pmc).  Summarise with
# tools/pmc_summary.py gpurun_out/$PMC_OUT.
PO=${PMC_OUT:-pmc}
mkdir -p gpurun_out/$PO
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/$PO
IFS=';' read -ra GRP <<< "${PMC_GROUPS:?}"
i=0
cd /tmp
for g in "${GRP[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d $R/pass_$i -o run -- \
      python3 $GRAFT_REPO_ROOT/$PMC_CMD > $R/pass_$i.log 2>&1 || exit $?
  i=$((i+1))
done
exit 0
