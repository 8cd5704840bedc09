"""Per-kernel duration and HBM traffic of one bench step from
tools/gpu_pmc_all.sh output: kernel trace + FETCH_SIZE / WRITE_SIZE passes
(KB units; FETCH_SIZE x2 as the gfx950 correction used for the bench's
roofline traffic)."""
import collections
import csv
import json
import os
import sys

root = sys.argv[1]
d = json.load(open(os.path.join(root, "pmc_summary.json")))
dur = collections.defaultdict(list)
for r in csv.DictReader(open(os.path.join(root, "kt", "kt_kernel_trace.csv"))):
    n = r["Kernel_Name"]
    k = "k_ms_walk2" if "ms_walk2" in n else "k_counter_win" if "counter_win" in n else n[:60]
    dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
rows = []
for k, v in d.items():
    f = v.get("FETCH_SIZE", {}).get("total", 0) * 2 * 1024 / 1e9
    w = v.get("WRITE_SIZE", {}).get("total", 0) * 1024 / 1e9
    rows.append((sum(dur.get(k, [0])), k, len(dur.get(k, [])), f, w))
rows.sort(reverse=True)
print("%-60s %4s %8s %9s %9s %7s" % ("kernel", "n", "ms", "fetch GB", "write GB", "GB/s"))
for t, k, n, f, w in rows:
    print("%-60s %4d %8.2f %9.3f %9.3f %7.0f" % (k, n, t, f, w, (f + w) / (t / 1e3) if t else 0))
