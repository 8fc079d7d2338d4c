"""Print the top kernels of a rocprofv3 --stats CSV (name, calls, avg us, %)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
for r in rows[:n]:
    print(f"{r['Name'][:80]:80s} {r['Calls']:>5s} {float(r['AverageNs']) / 1e3:10.1f}us {float(r['Percentage']):6.2f}")
