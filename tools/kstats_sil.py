"""Print the silhouette rows of every kernel_stats.csv under a directory (tools only)."""
import csv
import glob
import sys

for f in sorted(glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)):
    print(f)
    for r in csv.DictReader(open(f)):
        if any(t in r["Name"] for t in sys.argv[2:] or ["sil"]):
            print("   ", r["Name"][:50].ljust(50), r["Calls"], "%.1f us" % (float(r["AverageNs"]) / 1e3))
