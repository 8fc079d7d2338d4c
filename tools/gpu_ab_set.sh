# A/B of variant builds on one launch set (tools/set_micro.py): default, then each variant, twice
set -o pipefail
R=gpurun_out/${OUT:-abset}; mkdir -p $R
for rep in 1 2; do
  for v in default ${AB_VARIANTS}; do
    if [ $v = default ]; then L=""; else L="--lib tools/variants/libccg_$v.so"; fi
    timeout -k 10 150 python tools/set_micro.py $L > $R/set_${v}_$rep.json 2> $R/set_${v}_$rep.err || exit $?
  done
done
