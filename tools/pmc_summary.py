"""Summarise rocprofv3 --pmc passes (p*/p*_counter_collection.csv under a
directory) per kernel: counter totals over dispatches and per launch."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
per = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in sorted(glob.glob(os.path.join(root, "p*", "p*_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        key = ("k_ms_walk2" if "ms_walk2" in name else "k_counter_tgt" if "counter_tgt" in name
               else "k_counter_win" if "counter_win" in name else name[:60])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(key, r["Counter_Name"])].add(r["Dispatch_Id"])
out = {}
for k, d in per.items():
    out[k] = {c: {"total": v, "launches": len(disp[(k, c)]), "per_launch": v / max(1, len(disp[(k, c)]))}
              for c, v in sorted(d.items())}
json.dump(out, sys.stdout, indent=1)
