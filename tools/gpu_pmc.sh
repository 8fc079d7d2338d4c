#!/bin/bash
# PMC passes (each its own run, kernel-trace only) over the kNN micro-benchmark.
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/pmc/counters.txt 2>&1 || true
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES"; do
  tag=$(echo $set | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc/$tag -o run -- \
      python3 $GRAFT_REPO_ROOT/tools/knn_micro.py > $GRAFT_REPO_ROOT/gpurun_out/pmc/$tag.log 2>&1 || echo "pass $tag rc=$?" >> $GRAFT_REPO_ROOT/gpurun_out/pmc/fail.txt
done
exit 0
