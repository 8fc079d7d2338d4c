#!/bin/bash
# SNN micro-benchmark variants + kernel trace + one PMC pass.
mkdir -p gpurun_out/snn
export TMPDIR=/tmp
: > gpurun_out/snn/micro.log
for v in 0 1 2 3; do
  CCG_SNN_EXP=$v timeout -k 10 300 python tools/snn_micro.py >> gpurun_out/snn/micro.log 2>>gpurun_out/snn/micro.err || exit $?
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/snn/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/snn_micro.py > $GRAFT_REPO_ROOT/gpurun_out/snn/prof.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_INST_LDS \
    --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/snn/pmc/A -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/snn_micro.py > $GRAFT_REPO_ROOT/gpurun_out/snn/pmcA.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY \
    --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/snn/pmc/B -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/snn_micro.py > $GRAFT_REPO_ROOT/gpurun_out/snn/pmcB.log 2>&1 || exit $?
