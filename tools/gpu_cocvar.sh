mkdir -p gpurun_out; export TMPDIR=/tmp; : > gpurun_out/variants.log
for B in 125 1000; do for v in ${COCV:-base pipe}; do
  echo -n "B=$B $v " >> gpurun_out/variants.log
  CM_B=$B timeout -k 10 300 python tools/coc_micro.py --lib tools/variants/libccg_$v.so >> gpurun_out/variants.log 2>>gpurun_out/variants.err || exit $?
done; done
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread -k "cocluster or consensus or hierarchy or group or cfg4" > gpurun_out/pytest_gpu.log 2>&1
