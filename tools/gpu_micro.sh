#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/micro.log
timeout -k 10 300 python tools/knn_micro.py >> gpurun_out/micro.log 2>>gpurun_out/micro.err || exit $?
CCG_KNN_EXP=1 timeout -k 10 300 python tools/knn_micro.py >> gpurun_out/micro.log 2>>gpurun_out/micro.err || exit $?
CCG_KNN_F32=1 timeout -k 10 300 python tools/knn_micro.py >> gpurun_out/micro.log 2>>gpurun_out/micro.err || exit $?
