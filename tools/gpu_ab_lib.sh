# bench A/B of variant builds (CCG_LIB_PATH), interleaved: WLS workloads x (default + AB_VARIANTS)
set -o pipefail
R=$GRAFT_REPO_ROOT/gpurun_out/${OUT:-ablib}; mkdir -p $R
for w in ${WLS:-cfg5 cfg3}; do
  for v in default ${AB_VARIANTS}; do
    if [ $v = default ]; then L=""; else L=$GRAFT_REPO_ROOT/tools/variants/libccg_$v.so; fi
    CCG_LIB_PATH=$L timeout -k 10 400 python bench.py --workload $w --steps ${BSTEPS:-5} --warmup 1 --no-cpu-baseline > $R/${w}_$v.json 2> $R/${w}_$v.err || exit $?
  done
done
