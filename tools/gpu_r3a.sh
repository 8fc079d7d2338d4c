#!/bin/bash
# Round-3 checkpoint: kNN screen variants (tools/gpu_kexp.sh), the consensus
# kNN paths against the co-cluster triangle, the GPU tests touched this round,
# then a short bench.  Stops at the first failing step.
mkdir -p gpurun_out/r3a
export TMPDIR=/tmp
R=gpurun_out/r3a
VARIANTS="${VARIANTS:-base pair3 pair2 sonly nocand nomax pair2so}" bash tools/gpu_kexp.sh || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider -rf \
    --timeout 180 --timeout-method thread > $R/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $R/pytest.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python tools/cknn_micro.py > $R/cknn.json 2> $R/cknn.err || exit $?
timeout -k 10 300 python tools/pca_micro.py > $R/pca.json 2> $R/pca.err || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/bench.json 2> $R/bench.err || exit $?
