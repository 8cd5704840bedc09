# Per-kernel fabric traffic of one bench step (through gpurun from the repo
# root): FETCH_SIZE, WRITE_SIZE and the L2->fabric request counts of every
# kernel, one counter group per rocprofv3 run (no traces with --pmc).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/mpmc; rm -rf $OUT; mkdir -p $OUT
B1="python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --no-check"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $grp -d $OUT/p$i -o p$i --output-format csv -- $B1 > $OUT/p$i.log 2>&1
done
python3 tools/pmc_main.py $OUT > $OUT/pmc_main.json
python3 - "$OUT/pmc_main.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
rows = []
for k, v in d.items():
    if not isinstance(v, dict) or "FETCH_SIZE" not in v:
        continue
    rows.append((2 * v.get("FETCH_SIZE", 0) / 1e6 + v.get("WRITE_SIZE", 0) / 1e6, k, v))
rows.sort(reverse=True)
print("%-62s %8s %8s %9s %9s" % ("kernel (largest dispatch)", "fetchGB", "writeGB", "rdreq M", "wrreq M"))
for t, k, v in rows[:30]:
    print("%-62s %8.2f %8.2f %9.1f %9.1f" % (k[:62], 2 * v.get("FETCH_SIZE", 0) / 1e6, v.get("WRITE_SIZE", 0) / 1e6,
                                            v.get("TCC_EA0_RDREQ_sum", 0) / 1e6, v.get("TCC_EA0_WRREQ_sum", 0) / 1e6))
PY
