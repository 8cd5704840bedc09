"""L2 counters of the largest k_ms_walk2 / k_counter_tgt dispatch in a rocprofv3 --pmc directory."""
import csv, glob, sys

files = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)
per = {}
for r in csv.DictReader(open(files[0])):
    for k in ("k_ms_walk2", "k_counter_tgt"):
        if k in r["Kernel_Name"]:
            d = per.setdefault(k, {}).setdefault(r["Dispatch_Id"], {})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0) + float(r["Counter_Value"])
for k, ds in per.items():
    d = max(ds.values(), key=lambda x: x.get("TCC_MISS_sum", x.get("SQ_WAVE_CYCLES", 0)))
    print("variant", sys.argv[2], k, {c: f"{v:.3e}" for c, v in sorted(d.items())})
