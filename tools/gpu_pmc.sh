#!/bin/bash
# PMC passes (each its own run, kernel-trace only) over a micro-benchmark.
# PMC_PROG: the python program (default tools/knn_micro.py); PMC_TAG: output dir name.
mkdir -p gpurun_out
export TMPDIR=/tmp
PROG=${PMC_PROG:-tools/knn_micro.py}
OUT=$GRAFT_REPO_ROOT/gpurun_out/${PMC_TAG:-pmc}
mkdir -p $OUT
cd /tmp
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"; do
  tag=$(echo $set | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/$tag -o run -- \
      python3 $GRAFT_REPO_ROOT/$PROG > $OUT/$tag.log 2>&1 || { echo "pass $tag rc=$?" >> $OUT/fail.txt; exit 1; }
done
exit 0
