#!/bin/bash
# Round-6 evidence on the final tree, each step under its own limit, stop at
# the first failure.  Output: gpurun_out/$OUT.
#   bench lines of every workload (cfg3 with the CPU baseline + oracle check),
#   the default bench under rocprofv3 --kernel-trace --stats,
#   PMC passes (FETCH_SIZE; WRITE_SIZE; SQ) over one launch set (tools/set_micro.py),
#   the consensus-kNN micro (f1).
OUT=${OUT:-fin6}
R=$GRAFT_REPO_ROOT/gpurun_out/$OUT
mkdir -p $R
export TMPDIR=/tmp
echo "$(date +%T) start" > $R/progress.log
for w in ${WLS:-cfg3 cfg3job cfg2 cfg4 cfg5}; do
  X="--no-cpu-baseline"; [ $w = cfg3 ] && X=""
  echo "$(date +%T) bench $w" >> $R/progress.log
  timeout -k 10 ${BT:-420} python bench.py --workload $w --steps ${BSTEPS:-5} --warmup 1 $X \
      > $R/bench_$w.json 2> $R/bench_$w.err || exit $?
done
if [ -z "$NO_PROF" ]; then
  echo "$(date +%T) stats" >> $R/progress.log
  cd /tmp
  timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $R/stats -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/prof_bench.json 2> $R/prof.log \
      || exit $?
  echo "$(date +%T) set trace" >> $R/progress.log
  SM_REPS=1 timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $R/set_trace -o run -- \
      python3 $GRAFT_REPO_ROOT/tools/set_micro.py > $R/set_trace.log 2>&1 || exit $?
  i=0
  for g in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"; do
    echo "$(date +%T) pmc $g" >> $R/progress.log
    SM_REPS=1 timeout -s KILL 150 rocprofv3 --pmc $g --output-format csv -d $R/pmc/pass_$i -o run -- \
        python3 $GRAFT_REPO_ROOT/tools/set_micro.py > $R/pmc_$i.log 2>&1 || exit $?
    i=$((i+1))
  done
  cd $GRAFT_REPO_ROOT
fi
if [ -z "$NO_MICRO" ]; then
  echo "$(date +%T) cknn" >> $R/progress.log
  timeout -k 10 300 python tools/cknn_micro.py > $R/cknn_micro.json 2> $R/cknn_micro.err || exit $?
fi
if [ -z "$NO_E2E" ]; then
  echo "$(date +%T) e2e" >> $R/progress.log
  timeout -k 10 400 python tools/e2e_cfg2.py > $R/e2e_cfg2.json 2> $R/e2e_cfg2.err || exit $?
fi
echo "$(date +%T) done" >> $R/progress.log
exit 0
