# one launch set (tools/set_micro.py): kernel stats + FETCH_SIZE and WRITE_SIZE passes
set -o pipefail
R=$GRAFT_REPO_ROOT/gpurun_out/${OUT:-setprof}; mkdir -p $R
export TMPDIR=/tmp
cd /tmp
SM_REPS=1 timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $R/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/set_micro.py > $R/trace.log 2>&1 || exit $?
i=0
for g in FETCH_SIZE WRITE_SIZE; do
  SM_REPS=1 timeout -s KILL 150 rocprofv3 --pmc $g --output-format csv -d $R/pmc/pass_$i -o run -- python3 $GRAFT_REPO_ROOT/tools/set_micro.py > $R/pmc_$i.log 2>&1 || exit $?
  i=$((i+1))
done
