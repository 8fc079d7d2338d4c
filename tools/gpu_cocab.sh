set -o pipefail
mkdir -p gpurun_out/cocab
for cfg in "125 2 40" "1000 2 40"; do
  set -- $cfg
  for v in new old; do
    if [ $v = new ]; then L=""; else L="--lib tools/variants/libccg_old.so"; fi
    CM_B=$1 CM_CLO=$2 CM_CHI=$3 timeout -k 10 120 python tools/coc_micro.py $L > gpurun_out/cocab/coc_${1}_${v}.json 2>&1 || exit $?
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_group.py tests/test_gpu_consensus_clust.py tests/test_gpu_edges.py > gpurun_out/cocab/pytest.log 2>&1
