"""End-to-end A/B of the cmsbwt CLI on the bench workload's FASTA files:
CMSBWT_OVERLAP_UPLOAD=1/0 interleaved, wall times and the CLI's stage line."""
import os
import subprocess
import sys
import tempfile
import time

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
build = os.path.join(root, "cms-bwt_amd", "build")
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
    pre = os.path.join(td, "w")
    subprocess.run([os.path.join(build, "gen_synth"), "10000000", "1000", "0.001", "4", pre], check=True,
                   stdout=subprocess.DEVNULL)
    walls = {"1": [], "0": []}
    for _ in range(reps):
        for ov in ("1", "0"):
            env = dict(os.environ, CMSBWT_OVERLAP_UPLOAD=ov)
            t0 = time.perf_counter()
            r = subprocess.run([os.path.join(build, "cmsbwt"), "-r", "-v", "-o", pre + "_out", pre + ".list"],
                               env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True, timeout=120)
            w = time.perf_counter() - t0
            if r.returncode:
                sys.exit(f"cmsbwt exit {r.returncode}: {r.stderr[-300:]}")
            walls[ov].append(w)
            print(f"overlap={ov} wall={w:.3f} {r.stderr.strip().splitlines()[-1]}", flush=True)
    for ov, v in walls.items():
        print(f"overlap={ov} median {sorted(v)[len(v) // 2]:.3f} s  walls {[round(x, 3) for x in v]}")
