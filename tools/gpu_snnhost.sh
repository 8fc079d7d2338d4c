# SNN drop-in host decode: tests, then its timing in the cfg3 bench line (phase times on stderr)
set -o pipefail
R=gpurun_out/${OUT:-snnhost}; mkdir -p $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_contracts.py tests/test_gpu_edges.py > $R/pytest.log 2>&1 || exit $?
CCG_SNN_HOST_PROFILE=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/bench.json 2> $R/bench.err || exit $?
grep -h "host_snn\|\[ccg snn host\]" $R/bench.err > $R/host_phases.txt || true
if [ -n "$JOB" ]; then timeout -k 10 300 python bench.py --workload cfg3job --steps 2 --warmup 1 --no-cpu-baseline > $R/bench_cfg3job.json 2> $R/bench_cfg3job.err || exit $?; fi
if [ -n "$E2E" ]; then timeout -k 10 400 python tools/e2e_cfg2.py > $R/e2e_cfg2.json 2> $R/e2e_cfg2.err || exit $?; fi
