#!/bin/bash
# A/B bench runs (environment variants in AB_ENVS, ';'-separated) and a
# rocprofv3 --kernel-trace --stats run of bench.py $PROF_ARGS.  Each step has
# its own time limit; stops at the first failure.
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/prof
IFS=';' read -ra ENVS <<< "${AB_ENVS:-}"
i=0
for e in "${ENVS[@]}"; do
  env $e timeout -k 10 300 python bench.py --steps ${BSTEPS:-5} --warmup 2 --no-cpu-baseline ${BENCH_EXTRA:-} \
      > $R/ab_$i.json 2> $R/ab_$i.err || exit $?
  echo "$e" > $R/ab_$i.env
  i=$((i+1))
done
if [ -n "$PROF_ARGS" ]; then
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/stats -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py $PROF_ARGS > $R/prof.log 2>&1 || exit $?
fi
exit 0
