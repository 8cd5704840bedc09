"""End-to-end A/B of the cmsbwt CLI on the bench workload's FASTA files:
one environment variable's values interleaved, wall times, the CLI's stage
line and the output's checksum (all settings must write the same .rl_bwt).

  python tools/e2e_ab.py [reps] [VAR v1 v2 ...]
  (default: CMSBWT_OVERLAP_UPLOAD 1 0)"""
import hashlib
import os
import subprocess
import sys
import tempfile
import time

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
build = os.path.join(root, "cms-bwt_amd", "build")
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
var, vals = (sys.argv[2], sys.argv[3:]) if len(sys.argv) > 3 else ("CMSBWT_OVERLAP_UPLOAD", ["1", "0"])
with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
    pre = os.path.join(td, "w")
    subprocess.run([os.path.join(build, "gen_synth"), "10000000", "1000", "0.001", "4", pre], check=True,
                   stdout=subprocess.DEVNULL)
    walls = {v: [] for v in vals}
    sums = set()
    for _ in range(reps):
        for v in vals:
            env = dict(os.environ, **{var: v})
            t0 = time.perf_counter()
            r = subprocess.run([os.path.join(build, "cmsbwt"), "-r", "-v", "-o", pre + "_out", pre + ".list"],
                               env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True, timeout=120)
            w = time.perf_counter() - t0
            if r.returncode:
                sys.exit(f"cmsbwt exit {r.returncode}: {r.stderr[-300:]}")
            walls[v].append(w)
            with open(pre + "_out.rl_bwt", "rb") as f:
                sums.add(hashlib.sha256(f.read()).hexdigest()[:16])
            print(f"{var}={v} wall={w:.3f} {' '.join(r.stderr.strip().splitlines()[-2:])}", flush=True)
    for v, x in walls.items():
        print(f"{var}={v} median {sorted(x)[len(x) // 2]:.3f} s  walls {[round(y, 3) for y in x]}")
    print("outputs identical" if len(sums) == 1 else f"OUTPUTS DIFFER: {sorted(sums)}")
