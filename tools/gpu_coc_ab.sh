#!/bin/bash
# Co-cluster A/B: the co-cluster parity tests, then tools/coc_micro.py at
# B = 32 / 125 / 1000 with the default build and each variant given.
mkdir -p gpurun_out/cocab
R=gpurun_out/cocab
timeout -k 10 400 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -x \
    -k "cocluster or consensus or hierarchy or group" > $R/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $R/pytest.log
[ $rc -ne 0 ] && exit $rc
for B in 32 125 1000; do
  CM_B=$B timeout -k 10 200 python tools/coc_micro.py > $R/base_B$B.log 2>&1 || exit $?
  for v in "$@"; do
    CM_B=$B timeout -k 10 200 python tools/coc_micro.py --lib tools/variants/libccg_$v.so > $R/${v}_B$B.log 2>&1 || exit $?
  done
done
