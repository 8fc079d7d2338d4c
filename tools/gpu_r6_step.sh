#!/bin/bash
# Round-6 validation step: every -m gpu test (stop at the first failure),
# the co-cluster micro with the wide-tile kernel against the 128 x 256 one,
# then the bench A/B list (tools/gpu_ab_r6.sh).  Each step under its own
# limit.  Output: gpurun_out/$OUT.
OUT=${OUT:-r6s}
R=$GRAFT_REPO_ROOT/gpurun_out/$OUT
mkdir -p $R
export TMPDIR=/tmp
if [ "${PYTEST_K:-all}" != "none" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 180 --timeout-method thread -x \
      -k "${PYTEST_K:-not nothing}" > $R/pytest_gpu.log 2>&1 || exit $?
fi
for cfg in ${COC:-"125 30 44" "1000 2 40"}; do
  set -- $cfg
  for w in 1 0; do
    CCG_COF_WIDE=$w CM_B=$1 CM_CLO=$2 CM_CHI=$3 timeout -k 10 120 python tools/coc_micro.py \
        > $R/coc_${1}_${2}_w${w}.json 2>&1 || exit $?
  done
done
if [ -n "$AB" ]; then OUT=$OUT bash tools/gpu_ab_r6.sh || exit $?; fi
exit 0
