#!/bin/bash
# SNN parity tests + micro-benchmark variants.
mkdir -p gpurun_out/snn
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 -rf -k "snn or smoke or pipeline" > gpurun_out/snn/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/snn/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
: > gpurun_out/snn/micro.log
for v in ${SNN_VARIANTS:-0}; do
  CCG_SNN_EXP=$v timeout -k 10 300 python tools/snn_micro.py >> gpurun_out/snn/micro.log 2>>gpurun_out/snn/micro.err || exit $?
done
