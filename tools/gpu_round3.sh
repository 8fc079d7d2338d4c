#!/bin/bash
# Round-3 evidence: the whole GPU suite, the default bench (with the CPU
# baseline), rocprofv3 kernel stats of the default bench and of the
# single-stream variant, the co-cluster FETCH/WRITE PMC passes (traffic), and
# the micros for the fused consensus kNN (f1), the PCA (f4) and the co-cluster
# at B = 1000.  Stops at the first crash-like exit.
mkdir -p gpurun_out/r3
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/r3
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf \
    > $R/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $R/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > $R/bench.json 2> $R/bench.err || exit $?
timeout -k 10 200 python tools/cknn_micro.py > $R/cknn.json 2> $R/cknn.err || exit $?
timeout -k 10 200 python tools/pca_micro.py > $R/pca.json 2> $R/pca.err || exit $?
CM_B=1000 timeout -k 10 200 python tools/coc_micro.py > $R/coc_B1000.json 2> $R/coc_B1000.err || exit $?
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_default -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $R/prof_default.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_streams1 -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --streams 1 --boots-per-gpu 32 > $R/prof_streams1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_pca -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/pca_micro.py > $R/prof_pca.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  CM_B=125 CM_CLO=30 CM_CHI=44 timeout -k 10 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $R/pmc/$c -o run -- \
      python3 $GRAFT_REPO_ROOT/tools/coc_micro.py > $R/pmc_$c.log 2>&1 || exit $?
done
exit 0
