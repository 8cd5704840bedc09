"""Per-launch durations of the walk and counter kernels from a rocprofv3
kernel_trace.csv (tools/gpu_prof_r.sh).  The first k_ms_walk2 launch of an
engine is the head-density sample (a short prefix of the chunks, engine.h
ms_walk); the full launches are the ones bench.py times."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for key in ("k_ms_walk2", "k_counter_tgt"):
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows if key in r["Kernel_Name"]]
    full = d[1:] if key == "k_ms_walk2" and len(d) > 1 else d
    print(f"{key}: launches (ms) {' '.join(f'{x:.3f}' for x in d)}")
    print(f"{key}: average of the full launches {sum(full) / len(full):.3f} ms over {len(full)}"
          + (" (launch 1 = density sample, excluded)" if full is not d else ""))
