#!/bin/bash
# End-of-round check on the final tree: the whole GPU suite, smoke(), the default bench.
mkdir -p gpurun_out/fin
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/fin
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
    > $R/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $R/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $R/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $R/bench.json 2> $R/bench.err || exit $?
