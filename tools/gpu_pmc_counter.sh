# One SQ counter pass over the default bench; prints the counter kernels' values (through gpurun)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmcc
rm -rf $OUT; mkdir -p $OUT
B="python3 bench.py --steps 1 --warmup 0 --no-cpu"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT -d $OUT/p1 -o p1 --output-format csv -- $B > $OUT/p1.log 2>&1
python3 - <<'PY'
import csv,glob,collections
v=collections.defaultdict(dict)
for f in glob.glob("gpurun_out/pmcc/p1/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "counter_" in r["Kernel_Name"]:
            k=r["Kernel_Name"][:40]+"#"+r["Dispatch_Id"]
            v[k][r["Counter_Name"]]=float(r["Counter_Value"])
for k,d in v.items(): print(k, {a:f"{b:.3e}" for a,b in sorted(d.items())})
PY
