# kernel stats of one workload on the round-5 tree and on this tree
set -o pipefail
R=$GRAFT_REPO_ROOT/gpurun_out/prof_r05cmp; mkdir -p $R
W=${WL:-cfg5}
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT/tools/variants/r05
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/r05 -o run -- python3 bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline > $R/r05.json 2> $R/r05.err || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/cur -o run -- python3 bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline > $R/cur.json 2> $R/cur.err || exit $?
