#!/bin/bash
# Co-cluster entry-matrix loader: every co-cluster / consensus-kNN GPU test,
# tools/coc_micro.py at B = 125 and 1000, then the bench.
mkdir -p gpurun_out/ce
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/ce
timeout -k 10 600 python -u -m pytest tests/test_gpu_edges.py tests/test_gpu_parity.py tests/test_gpu_baseline_shapes.py \
    tests/test_gpu_group.py tests/test_gpu_hierarchy.py tests/test_gpu_pipeline.py tests/test_gpu_scale.py \
    -q -x -p no:cacheprovider -rf --timeout 300 --timeout-method thread > $R/pytest.log 2>&1 || exit $?
timeout -k 10 200 python tools/coc_micro.py > $R/coc_B125.log 2>&1 || exit $?
CM_B=1000 timeout -k 10 200 python tools/coc_micro.py > $R/coc_B1000.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/bench.json 2> $R/bench.err || exit $?
