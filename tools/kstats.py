"""Print a rocprofv3 kernel_stats.csv as a short table (ms per kernel)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows:
    print(f"{float(r['TotalDurationNs']) / 1e6:8.2f} ms {int(r['Calls']):4d}  {r['Name'][:100]}")
print(f"total {tot / 1e6:.2f} ms")
