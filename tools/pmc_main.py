"""Per-kernel PMC values of the main dispatch (the one with the most waves /
the largest counter total) from rocprofv3 --pmc passes under a directory;
FETCH_SIZE/WRITE_SIZE are in KiB (rocprofv3 derived counters)."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(dict))  # kernel -> counter -> dispatch -> value
for f in sorted(glob.glob(os.path.join(root, "p*", "p*_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        key = ("k_ms_walk2" if "ms_walk2" in name else "k_counter_tgt" if "counter_tgt" in name
               else "k_counter_win" if "counter_win" in name else name[:60])
        vals[key][r["Counter_Name"]][r["Dispatch_Id"]] = float(r["Counter_Value"])
out = {}
for k, cs in vals.items():
    # the main dispatch of each pass: the largest value of that pass's counter
    out[k] = {c: max(d.values()) for c, d in sorted(cs.items())}
    out[k]["_note"] = "largest dispatch per counter pass (the full launch, not the density-sample walk)"
json.dump(out, sys.stdout, indent=1)
