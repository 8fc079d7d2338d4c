"""Summarise a rocprofv3 kernel_stats.csv: share, calls, average per kernel."""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
pat = sys.argv[3] if len(sys.argv) > 3 else ""
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    if pat and pat not in r["Name"]:
        continue
    print(f"{float(r['TotalDurationNs']) / tot * 100:6.2f}% {int(r['Calls']):7d} {float(r['AverageNs']) / 1e3:9.1f}us {r['Name'][:95]}")
    n -= 1
    if n == 0:
        break
print(f"total {tot / 1e6:.1f} ms")
