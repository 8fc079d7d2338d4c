#!/bin/bash
# Cell-table kNN, radius exact search, SNN copy nodes, distinct-cell
# silhouette: the whole GPU suite, the silhouette micro, both bench kNN paths,
# and a kernel-stats profile of the default bench.
mkdir -p gpurun_out/tab
export TMPDIR=/tmp
R=gpurun_out/tab
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider -rf \
    --timeout 180 --timeout-method thread > $R/pytest.log 2>&1 || exit $?
timeout -k 10 200 python tools/sil_micro.py > $R/sil.json 2> $R/sil.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $R/bench_table.json 2> $R/bench_table.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --knn-path screen > $R/bench_screen.json 2> $R/bench_screen.err || exit $?
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$R/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/$R/prof.log 2>&1 || exit $?
