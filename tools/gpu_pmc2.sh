#!/bin/bash
# PMC passes (one rocprofv3 run per counter set) over a micro-benchmark.
#   PMC_PROG     : script under tools/ (default knn_micro.py)
#   PMC_VARIANTS : values of $PMC_ENV (default CCG_KNN_EXP) to profile, one pass set each
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
prog=${PMC_PROG:-knn_micro.py}
envn=${PMC_ENV:-CCG_KNN_EXP}
cd /tmp
for v in ${PMC_VARIANTS:-0}; do
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
           "SQ_ACTIVE_INST_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_LDS_IDX_ACTIVE SQ_INSTS_FLAT"; do
  tag=v${v}_$(echo $set | cut -d' ' -f1)
  export $envn=$v; timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc2/$tag -o run -- \
      python3 $GRAFT_REPO_ROOT/tools/$prog > $GRAFT_REPO_ROOT/gpurun_out/pmc2/$tag.log 2>&1 || echo "pass $tag rc=$?" >> $GRAFT_REPO_ROOT/gpurun_out/pmc2/fail.txt
done
done
exit 0
