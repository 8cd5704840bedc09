"""Dispatch-by-dispatch timeline of the last step in a rocprofv3 kernel_trace.csv
(tools/gpu_kt.sh): consecutive launches of the same kernel are merged."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last step starts at the last k_ms_walk2 launch
starts = [i for i, r in enumerate(rows) if "k_ms_walk2" in r["Kernel_Name"]]
rows = rows[starts[-1]:]
t0 = int(rows[0]["Start_Timestamp"])
out = []
for r in rows:
    name = r["Kernel_Name"]
    short = name.split("(")[0].replace("void ", "")
    if "rocprim" in name:
        short = "rocprim:" + ("lookback" if "lookback" in name else "sort" if "sort" in name else
                             "scan" if "scan" in name else "select" if "select" in name else
                             "reduce" if "reduce" in name else "other")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    s = (int(r["Start_Timestamp"]) - t0) / 1e6
    if out and out[-1][0] == short:
        out[-1][1] += d
        out[-1][3] += 1
    else:
        out.append([short, d, s, 1])
tot = 0
for name, d, s, c in out:
    tot += d
    print(f"{s:9.2f} {d:8.3f} ms x{c:<3d} {name[:90]}")
end = max(int(r["End_Timestamp"]) for r in rows)
print(f"busy {tot:.2f} ms, span {(end - t0) / 1e6:.2f} ms")
