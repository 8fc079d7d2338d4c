# A/B of library variants on the isolated per-bootstrap chain (tools/boot_micro.py)
mkdir -p gpurun_out/ab
for v in default ${AB_VARIANTS:-}; do
  if [ $v = default ]; then L=""; else L="--lib tools/variants/libccg_$v.so"; fi
  BM_BOOTS=${BM_BOOTS:-16} timeout -k 10 200 python tools/boot_micro.py $L > gpurun_out/ab/boot_${v}.json 2>&1 || exit $?
done
