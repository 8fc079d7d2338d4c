# cfg5 regression hunt: the round-5 tree (worktree in tools/variants/r05) against this tree, interleaved
set -o pipefail
R=$GRAFT_REPO_ROOT/gpurun_out/ab_r05; mkdir -p $R
W=${WL:-cfg5}
for rep in 1 2; do
  (cd tools/variants/r05 && timeout -k 10 300 python bench.py --workload $W --steps 5 --warmup 1 --no-cpu-baseline > $R/r05_${W}_$rep.json 2> $R/r05_${W}_$rep.err) || exit $?
  timeout -k 10 300 python bench.py --workload $W --steps 5 --warmup 1 --no-cpu-baseline > $R/cur_${W}_$rep.json 2> $R/cur_${W}_$rep.err || exit $?
done
