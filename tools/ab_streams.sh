# bench.py at several bootstraps-in-flight counts (cfg3, no CPU baseline)
mkdir -p gpurun_out/ab
for s in ${STREAMS:-2 3 4}; do
  timeout -k 10 300 python bench.py --steps ${BSTEPS:-5} --warmup 2 --no-cpu-baseline --streams $s \
      > gpurun_out/ab/streams_$s.json 2> gpurun_out/ab/streams_$s.err || exit $?
done
