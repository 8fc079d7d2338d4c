# bench lines of the named workloads (default cfg5 cfg3), 5 steps each
set -o pipefail
R=$GRAFT_REPO_ROOT/gpurun_out/${OUT:-quick}; mkdir -p $R
for w in ${WLS:-cfg5 cfg3}; do
  timeout -k 10 400 python bench.py --workload $w --steps ${BSTEPS:-5} --warmup 1 --no-cpu-baseline > $R/bench_$w.json 2> $R/bench_$w.err || exit $?
done
