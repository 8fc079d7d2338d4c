mkdir -p gpurun_out/ab
for cfg in "125 2 40" "125 30 44" "1000 2 40"; do
  set -- $cfg
  for v in default ${AB_VARIANTS:-}; do
    if [ $v = default ]; then L=""; else L="--lib tools/variants/libccg_$v.so"; fi
    CM_B=$1 CM_CLO=$2 CM_CHI=$3 timeout -k 10 120 python tools/coc_micro.py $L > gpurun_out/ab/coc_${1}_${2}_${v}.json 2>&1 || exit $?
  done
done
