#!/bin/bash
# bench.py at several --streams values (bootstraps in flight per GPU).
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/streams.log
for s in ${STREAMS:-2 3 4}; do
  echo -n "streams=$s " >> gpurun_out/streams.log
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --streams $s 2>>gpurun_out/streams.err \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" \
      >> gpurun_out/streams.log || exit $?
done
