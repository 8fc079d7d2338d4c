# HIP runtime API trace + kernel trace of a short bench of one workload (host-side stalls)
set -o pipefail
R=$GRAFT_REPO_ROOT/gpurun_out/hiptrace; mkdir -p $R
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --hip-runtime-trace --kernel-trace --output-format csv -d $R/t -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload ${WL:-cfg5} --steps 2 --warmup 1 --no-cpu-baseline > $R/b.json 2> $R/b.err || exit $?
cd $R/t && python3 - <<'PY'
import csv, glob, collections
f = glob.glob('**/run_hip_api_trace.csv', recursive=True)
rows = list(csv.DictReader(open(f[0])))
agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
for r in rows:
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
    a = agg[r['Function']]
    a[0] += 1; a[1] += d; a[2] = max(a[2], d)
with open('../api_summary.txt', 'w') as out:
    for k, v in sorted(agg.items(), key=lambda x: -x[1][1])[:40]:
        out.write(f"{v[0]:8d} {v[1]:10.2f} ms  max {v[2]:8.3f} ms  {k}\n")
PY
rm -f $R/t/*/run_hip_api_trace.csv $R/t/run_hip_api_trace.csv
