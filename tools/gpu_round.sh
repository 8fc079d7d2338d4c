#!/bin/bash
# Round-end evidence: GPU parity tests, the default bench (with the CPU
# baseline), rocprofv3 kernel stats of the default bench command and of the
# isolated (--streams 1) variant, and the FETCH/WRITE PMC passes of the kNN
# screen (traffic).  Stops at the first crash-like exit.
mkdir -p gpurun_out/round
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/round
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf \
    > $R/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $R/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > $R/bench.json 2> $R/bench.err || exit $?
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_default -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $R/prof_default.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_streams1 -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --streams 1 --boots-per-gpu 32 > $R/prof_streams1.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $R/pmc/$c -o run -- \
      python3 $GRAFT_REPO_ROOT/tools/knn_micro.py > $R/pmc_$c.log 2>&1 || exit $?
done
exit 0
