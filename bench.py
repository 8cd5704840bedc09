"""bench.py — collection MB/s of the CMS-BWT hot path on MI355X.

Workload (BASELINE.json configs[2]): one 10 MB synthetic DNA
reference + 1000 copies mutated at 0.1 % SNP rate (10 GB of collection text),
-r output.  The collection is generated directly in HBM by the same
counter-based generator as tools/gen_synth (synth.h), so the timed region
starts with inputs resident.  One step = MS walk + j-scan + the whole merge to
packed .rl_bwt run records in HBM (cmsbwt_step); the reference index is built
once before timing.

value = collection sequence bytes / 1e6 / seconds per step, whole job.

Two more legs ride on the same line (rank 0, N = 1):
* "e2e" — SURVEY.md §8(d) Metric 1: the `cmsbwt -r` process on FASTA files
  of the same workload written by the product's gen_synth (page cache), wall
  time from process start to output closed; the .rl_bwt's sha256 is compared
  with the oracle's golden for this workload (tests/golden/golden.json).
* "cpu_baseline" — the single-threaded CPU oracle on a bounded sample.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cms-bwt_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def synth_reference(L: int, seed: int) -> bytes:
    """Same bytes as synth.h: ref[k] = "ACGT"[h(seed, 0, k) >> 62]."""
    import numpy as np
    M = np.uint64(0xFFFFFFFFFFFFFFFF)

    def mix(z):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))

    with np.errstate(over="ignore"):
        s = mix(np.uint64(seed) + np.uint64(0xD1B54A32D192ED03) * np.uint64(1))
        k = np.arange(L, dtype=np.uint64)
        h = mix(s ^ k)
    del M
    return np.frombuffer(b"ACGT", dtype=np.uint8)[(h >> np.uint64(62)).astype(np.int64)].tobytes()


def host_cpu():
    """This host's CPU model and hardware threads (the CPU legs use one)."""
    model = ""
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = None
    return {"model": model, "threads_total": os.cpu_count(), "threads_available": avail, "threads_used": 1}


def cpu_baseline(ref_len, copies, p, seed, rle=True, full_copies=None):
    """Oracle (single-threaded CPU restatement) on a bounded sample of the same
    workload, collection stage only (parse .. .rl_bwt closed), timed on this
    host: that is `value`.  The counter phase grows with the copy count, so a
    short sample overstates the CPU's rate on the full workload; the oracle's
    own full-size run of this workload (timed once in the build container,
    tests/golden/golden.json) rides beside it as `full_workload`."""
    import oracle_lib
    gen = oracle_lib.GEN
    with tempfile.TemporaryDirectory() as td:
        pre = os.path.join(td, "s")
        subprocess.run([gen, str(ref_len), str(copies), str(p), str(seed), pre], check=True)
        rc, st, (t_idx, t_coll) = oracle_lib.run(pre + ".ref.fa", pre + ".coll.fa", pre + "_o", rle=rle)
        if rc:
            raise RuntimeError(f"oracle rc={rc}")
    chars = ref_len * copies
    out = {"value": round(chars / 1e6 / t_coll, 3), "unit": "MB/s", "cores": 1, "kind": "port", "host": host_cpu(),
           "sample": f"{ref_len // 10**6} MB ref + {copies} copies @{p * 100:g}% ({chars / 1e6:.0f} MB collection) "
                     f"of the bench workload's generator, oracle collection stage {t_coll:.2f} s on this host "
                     f"(one thread), index {t_idx:.2f} s excluded",
           "seconds": round(t_coll, 3)}
    full = golden_entry(ref_len, full_copies, p, seed) if full_copies else None
    if full and full.get("oracle_collection_seconds"):
        fs = full["oracle_collection_seconds"]
        fv = ref_len * full_copies / 1e6 / fs
        out["full_workload"] = {"value": round(fv, 3), "unit": "MB/s", "cores": 1, "seconds": fs,
                                "timed_on": "build container (8-vCPU Xeon), once (~28 min; tests/golden/golden.json)",
                                "sample": f"the whole workload ({full_copies} copies, "
                                          f"{ref_len * full_copies / 1e6:.0f} MB)"}
        out["sample_over_full"] = round(out["value"] / fv, 2)
    return out


PMC_FILE = "r06_final_pmc.json"  # tools/gpu_round_prof.sh: tools/gpu_prof_r.sh + tools/pmc_main.py (this round's kernels)

# Algorithmic bytes of the MS walk (k_ms_walk2) -- what THIS algorithm must
# move, each byte counted once (DESIGN.md §3.1 "Roofline"):
#   per collection character: the text byte and the reference byte it is
#     compared with at the extension frontier (FN:52-62); positions the PLCP
#     skip covers (FN:1176-1185) are compared once, by the extension that
#     reached them;
#   per head: its 16-B record (pool write), the 8-B prefix-table entry that
#     resolves it (one probe per head), and the 4-B PLCP entry at the skip exit.
WALK_B_PER_CHAR = 2
WALK_B_PER_HEAD = 16 + 8 + 4
# SURVEY.md §8(d)'s model prices the reference's per-character streams
# (1 B text + 1 B ref + 4 B PLCP + 16 B int64 bucket RMW per character, 24 B
# per head), which this walk replaces by run difference arrays and one skip
# per head; reported beside, as frac_survey_model.
SURVEY_B_PER_CHAR, SURVEY_B_PER_HEAD = 22, 24


def pmc_traffic(args, kernel="k_ms_walk2"):
    """Beyond-L2 bytes per launch of a kernel from the committed PMC summary
    (rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes, KiB units;
    tools/gpu_prof_r.sh), for the default workload only.  Per
    MI355X_MICROARCH.md (HBM): FETCH_SIZE = TCC_EA0_RDREQ x 64 B counts half
    the bytes of 128-B requests on gfx950, so it is doubled; both counters
    include Infinity-Cache hits, so this is fabric traffic, an upper bound on
    HBM bytes."""
    default = (args.ref_len, args.copies, args.p, args.seed) == (10_000_000, 1000, 0.001, 4)
    path = os.path.join(ROOT, "profiles", PMC_FILE)
    if not default or not os.path.exists(path):
        return None, None
    try:
        d = json.load(open(path))[kernel]
        b = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024.0
        return int(b), f"profiles/{PMC_FILE} (2 x FETCH_SIZE + WRITE_SIZE of the launch)"
    except (KeyError, ValueError, TypeError):
        return None, None


def golden_entry(ref_len, copies, p, seed):
    """The oracle's committed results for this exact synth.h workload, if any."""
    try:
        g = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
    except (OSError, ValueError):
        return None
    for k, v in g.items():
        if isinstance(v, dict) and v.get("generator") == "synth.h" and v.get("args") == [ref_len, copies, p, seed]:
            return v
    return None


def golden_for(args, rle):
    """The oracle's sha256 for this exact workload, when committed."""
    v = golden_entry(args.ref_len, args.copies, args.p, args.seed)
    return v.get("rl_bwt_sha256" if rle else "bwt_sha256") if v else None


def parity_check(eng, args, rle):
    """sha256 of the runs of the last timed step (rank 0 holds them) and the
    global statistics, against the oracle's golden for this workload."""
    import hashlib
    st = eng.stats()
    out = {"heads": st.heads, "keys": st.keys, "rank": st.rank, "runs": st.runs,
           "counter_bad": st.counter_bad, "counter_good": st.counter_good, "counter_nothing": st.counter_nothing}
    if not rle:
        out["verdict"] = "not checked (plain runs; the golden holds the expanded .bwt)"
        return out
    sha = hashlib.sha256(eng.runs_bytes()).hexdigest()
    out["rl_bwt_sha256"] = sha[:16]
    g = golden_entry(args.ref_len, args.copies, args.p, args.seed)
    if not g:
        out["verdict"] = "no golden for this workload"
        return out
    want = {"heads": g["headNumber"], "keys": g["keys"], "rank": g["Rank"], "runs": g["rl_runs"],
            "counter_bad": g["counterBad"], "counter_good": g["counterGood"], "counter_nothing": g["counterDoNothing"]}
    bad = [k for k, v in want.items() if out[k] != v]
    if sha != g["rl_bwt_sha256"]:
        bad.append("rl_bwt_sha256")
    out["verdict"] = "bit-exact vs oracle golden" if not bad else "MISMATCH vs oracle golden: " + ",".join(bad)
    return out


def _sha256_file(path):
    import hashlib
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 24), b""):
            h.update(blk)
    return h.hexdigest()


def e2e_leg(args, rle):
    """SURVEY.md §8(d) Metric 1: collection MB/s of the drop-in CLI, wall time
    from process start to output closed, on FASTA files in the page cache."""
    import shutil
    build = os.path.join(ROOT, "cms-bwt_amd", "build")
    gen, cli = os.path.join(build, "gen_synth"), os.path.join(build, "cmsbwt")
    base = os.environ.get("CMSBWT_E2E_DIR") or os.environ.get("TMPDIR") or "/tmp"
    chars = args.ref_len * args.copies
    need = int(chars * 1.05) + (chars // 8 if rle else chars) + (1 << 30)
    free = shutil.disk_usage(base).free
    if free < need:
        return {"skipped": f"{base} has {free >> 20} MiB free, needs {need >> 20} MiB"}
    td = tempfile.mkdtemp(prefix="cmsbwt_e2e_", dir=base)
    try:
        pre = os.path.join(td, "w")
        t0 = time.perf_counter()
        subprocess.run([gen, str(args.ref_len), str(args.copies), str(args.p), str(args.seed), pre], check=True)
        t_gen = time.perf_counter() - t0
        walls, stages = [], ""
        for _ in range(args.e2e_reps):
            cmd = [cli] + (["-r"] if rle else []) + ["-v", "-o", pre + "_out", pre + ".list"]
            t0 = time.perf_counter()
            r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
            walls.append(time.perf_counter() - t0)
            if r.returncode:
                return {"error": f"cmsbwt exit {r.returncode}: {r.stderr[-400:]}"}
            stages = " ".join(ln for ln in r.stderr.strip().splitlines() if ln.startswith(("context", "cli:")))
        out = pre + "_out" + (".rl_bwt" if rle else ".bwt")
        sha = _sha256_file(out)
        want = golden_for(args, rle)
        med = sorted(walls)[len(walls) // 2]
        return {"metric": "collection MB/s, cmsbwt process start to output closed (SURVEY.md §8d Metric 1)",
                "value": round(chars / 1e6 / med, 1), "unit": "MB/s", "wall_s": [round(w, 3) for w in walls],
                "wall_median_s": round(med, 3), "output_bytes": os.path.getsize(out),
                "stages": stages, "input": "FASTA files in the page cache (product gen_synth, %.1f s)" % t_gen,
                "sha256": sha[:16],
                "parity": ("bit-exact vs oracle golden" if want and sha == want else
                           "MISMATCH vs oracle golden" if want else "no golden for this workload")}
    finally:
        shutil.rmtree(td, ignore_errors=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--ref-len", type=int, default=10_000_000)
    ap.add_argument("--copies", type=int, default=1000)
    ap.add_argument("--p", type=float, default=0.001)
    ap.add_argument("--seed", type=int, default=4)
    ap.add_argument("--cpu-copies", type=int, default=30)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end CLI leg (Metric 1)")
    ap.add_argument("--no-check", action="store_true", help="skip the sha256 check of the last step's runs")
    ap.add_argument("--e2e-reps", type=int, default=3)
    ap.add_argument("--plain", action="store_true",
                    help="plain .bwt instead of .rl_bwt (BASELINE config 5 runs without -r)")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if env_world is not None and world != args.gpus:
        # the line's n_gpus must be the ranks that actually ran
        print(json.dumps({"error": f"--gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a "
                                   "number for a different rank count"}), flush=True)
        sys.exit(2)
    # --gpus N > 1 without a launcher: the product's in-process multi-GPU path
    # (multi.hip rank group: one host thread and context per rank, rank k on
    # device k % devices, the same walk + position-sharded merge as cmsbwt -n N)
    in_process = env_world is None and args.gpus > 1
    if in_process:
        world = args.gpus
    import torch
    # n_gpus is the number of distinct devices the ranks ran on: ranks that
    # would share a device (more in-process ranks than devices, or torchrun
    # ranks rehearsed on one GPU) are refused unless the rehearsal is asked
    # for explicitly, and then reported as ranks beside n_gpus (main.cpp:85-132
    # has no such mode)
    rehearsal = os.environ.get("CMSBWT_BENCH_REHEARSAL", "0") == "1"
    ndev = torch.cuda.device_count()  # (does not initialise the GPU on this image)
    if in_process and world > ndev and not rehearsal:
        print(json.dumps({"error": f"--gpus {world} in one process but {ndev} device(s): ranks would share a "
                                   "device; set CMSBWT_BENCH_REHEARSAL=1 to run them as a rehearsal "
                                   "(reported as n_gpus = distinct devices, ranks = N)"}), flush=True)
        sys.exit(2)
    dist = None
    # Rehearsal of the N>1 path on a one-GPU box (never set by the driver):
    # CMSBWT_BENCH_SAME_GPU=1 puts every rank on device 0 and uses gloo (host
    # staging) instead of RCCL, which allows one rank per device.
    same_gpu = os.environ.get("CMSBWT_BENCH_SAME_GPU", "0") == "1"
    if same_gpu:
        if world > 1 and not rehearsal:
            print(json.dumps({"error": "CMSBWT_BENCH_SAME_GPU=1 puts every rank on device 0; set "
                                       "CMSBWT_BENCH_REHEARSAL=1 as well (reported as n_gpus = 1, ranks = N)"}),
                  flush=True)
            sys.exit(2)
        local = 0
    if world > 1 and not in_process:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("gloo" if same_gpu else "nccl", init_method="env://")

    import cmsbwt
    import cmsbwt.dist as cdist
    ref = synth_reference(args.ref_len, args.seed)
    grp = None
    backend = os.environ.get("CMSBWT_BENCH_BACKEND", "peer")  # in-process transport: peer | rccl
    if in_process:
        grp = cmsbwt.Group(world, device=0, backend=backend)
        for k in range(world):
            e = grp.engine(k)
            e.load_reference_bytes(ref)
            c0, c1 = cdist.shard_range(args.copies, world, k)
            e.load_synth(args.seed, 1 + c0, c1 - c0, args.p, leading_empty_doc=(k == 0))
        eng = grp.engine(0)
    else:
        eng = cmsbwt.Engine(local)
        eng.load_reference_bytes(ref)
        # documents shard by contiguous ranges (the walk and j-scan are document-local)
        c0, c1 = cdist.shard_range(args.copies, world, rank)
        eng.load_synth(args.seed, 1 + c0, c1 - c0, args.p, leading_empty_doc=(rank == 0))
    device = f"cuda:{local}"
    mode = os.environ.get("CMSBWT_DIST", "sharded")  # N>1: sharded | gather; "sharded1": sharded path at N=1
    gather = mode == "gather"
    xfer = cdist.Transport(device) if ((world > 1 and not in_process) or mode == "sharded1") else None
    group_rows = []  # in-process: per-rank stage times of each timed step

    rle = not args.plain
    # per-step stage wall times of this rank (N > 1: walk, then the sharded
    # or gathered merge) and the walk statistics of this rank's shard
    stage = {"walk": 0.0, "merge": 0.0, "n": 0}
    walk_local = {}

    def step():
        if world == 1 and mode != "sharded1":
            eng.step(rle=rle)
            return
        if in_process:  # every rank's walk + the sharded merge, synchronous
            group_rows.append(grp.step(rle))
            return
        t0 = time.perf_counter()
        eng.ms_walk()  # synchronous: ends with the engine stream drained
        t1 = time.perf_counter()
        w = eng.stats()
        walk_local.update(heads=w.heads, chars=w.chars, kernel_ms=w.ms_walk_kernel_ms)
        if gather:    # all heads to rank 0, single-GPU merge there
            cdist.gather_merge(eng, device, rle=rle)
        else:         # merge sharded by reference position (dist_merge.hip)
            cdist.sharded_merge(eng, xfer, rle)
        stage["walk"] += t1 - t0
        stage["merge"] += time.perf_counter() - t1
        stage["n"] += 1

    def barrier():
        torch.cuda.synchronize(local)
        if dist:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    barrier()
    stage.update(walk=0.0, merge=0.0, n=0)
    group_rows.clear()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    dt = time.perf_counter() - t0
    st = eng.stats()
    if world == 1 and mode != "sharded1":
        walk_local.update(heads=st.heads, chars=st.chars, kernel_ms=st.ms_walk_kernel_ms)
        stage.update(walk=st.t_ms_walk_s * args.steps, merge=st.t_merge_s * args.steps, n=args.steps)
    ns = max(1, stage["n"])
    # per rank: [step time, walk stage, merge stage, walk kernel] -> max over
    # ranks; the walk roofline below is that of the slowest rank's kernel
    # (algorithmic bytes of the rank whose kernel was slowest)
    mine = None if in_process else [dt, stage["walk"] / ns, stage["merge"] / ns, walk_local["kernel_ms"],
                                    float(walk_local["heads"]), float(walk_local["chars"]),
                                    float(st.device_peak_bytes)]
    if dist:
        t = torch.tensor(mine, device="cpu" if same_gpu else f"cuda:{local}", dtype=torch.float64)
        allt = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allt, t)
        rows = [[float(v) for v in x.cpu().tolist()] for x in allt]
    elif in_process:  # one wall clock for the whole group; per-rank stage means
        K = max(1, len(group_rows))
        rows = [[dt] + [sum(getattr(s[k], f) for s in group_rows) / K / (1e3 if f != "walk_kernel_ms" else 1)
                        for f in ("walk_ms", "merge_ms", "walk_kernel_ms")] +
                [float(group_rows[-1][k].heads), float(group_rows[-1][k].chars),
                 float(group_rows[-1][k].device_peak_bytes)] for k in range(world)]
    else:
        rows = [mine]
    dt = max(r[0] for r in rows)
    slow = max(rows, key=lambda r: r[3])
    chars_total = args.ref_len * args.copies
    ms_step = dt / args.steps * 1e3
    value = chars_total / 1e6 / (dt / args.steps)

    # Roofline of the dominant kernel, the MS walk: algorithmic bytes of this
    # algorithm (WALK_B_PER_*) over its HIP-event duration (last step, on the
    # engine's stream, where the kernel is launched); N > 1: the slowest rank
    n_local, heads_local = int(slow[5]), int(slow[4])
    b_alg = WALK_B_PER_CHAR * n_local + WALK_B_PER_HEAD * heads_local
    b_survey = SURVEY_B_PER_CHAR * n_local + SURVEY_B_PER_HEAD * heads_local
    # compulsory HBM bytes if the 10 MB reference and every table stayed in
    # the caches: each text byte read once + each 16-B head record written
    b_floor = n_local + 16 * heads_local
    t_ms = slow[3] / 1e3
    achieved = b_alg / t_ms / 1e9 if t_ms > 0 else 0.0
    traffic, traffic_src = pmc_traffic(args) if world == 1 else (None, None)
    ctraffic, _ = pmc_traffic(args, "k_counter_tgt") if world == 1 else (None, None)
    c_ms = st.counter_kernel_ms
    # distinct devices the ranks ran on (the rehearsals share device 0)
    n_devices = 1 if same_gpu else min(world, ndev) if in_process else world
    out = {
        "metric": ("collection MB/s to .bwt" if args.plain else
                   "collection MB/s to .rl_bwt (10 MB ref + 1000 copies @0.1% SNP)"),
        "value": round(value, 3), "unit": "MB/s", "n_gpus": n_devices, "ranks": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (counter-based generator in HBM, SURVEY.md §8d)",
        "config": {"workload": f"{args.ref_len // 10**6} MB ref + {args.copies} copies @{args.p * 100:g}% SNP"
                               + ("" if args.plain else ", -r"),
                   "ref_len": args.ref_len, "copies": args.copies, "snp": args.p, "seed": args.seed,
                   "collection_bytes": chars_total, "heads": st.heads, "keys": st.keys, "runs": st.runs,
                   "parallelism": ((f"{world} in-process ranks (multi.hip rank group, rank k on device "
                                    f"k % {torch.cuda.device_count()}), {backend} transport; walk: documents "
                                    "sharded; merge: reference positions sharded, runs gathered to rank 0"
                                    if in_process else
                                    f"documents sharded over {world} GPUs, heads gathered to rank 0 over RCCL, merge on rank 0"
                                    if gather else
                                    f"walk: documents sharded over {world} GPUs; merge: reference positions sharded, "
                                    "all-to-all/all-reduce over RCCL, runs gathered to rank 0")
                                   if world > 1 else "1 GPU")},
        "roofline": {"bound": "hbm", "kernel": "k_ms_walk2", "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "algorithmic_bytes": b_alg, "kernel_ms": round(slow[3], 3),
                     "bytes_model": f"{WALK_B_PER_CHAR} B/char (text + reference byte at the extension frontier) "
                                    f"+ {WALK_B_PER_HEAD} B/head (16-B record, 8-B prefix probe, 4-B PLCP exit); "
                                    "DESIGN.md §3.1",
                     "traffic_over_algorithmic": round(traffic / b_alg, 2) if traffic else None,
                     "traffic_GBps": round(traffic / t_ms / 1e9, 1) if traffic and t_ms > 0 else None,
                     "hbm_floor_bytes": b_floor,
                     "frac_hbm_floor": round(b_floor / t_ms / 1e9 / HBM_PEAK_GBS, 4) if t_ms > 0 else None,
                     "hbm_floor_model": "1 B/char (text read once) + 16 B/head (record written): reference "
                                        "and tables assumed cache-resident",
                     "frac_survey_model": round(b_survey / t_ms / 1e9 / HBM_PEAK_GBS, 4) if t_ms > 0 else None,
                     "survey_model": "22 B/char + 24 B/head (SURVEY.md §8d: the reference's per-character "
                                     "streams; exceeds 1 because this walk does not perform them)"},
        # the merge's largest kernel (counterSmallerThanHead, FN:1523-1603):
        # register/LDS-bound, measured HBM traffic for reference
        "counter_kernel": {"kernel": "k_counter_tgt", "kernel_ms": round(c_ms, 3),
                           "queries": int(st.counter_good + st.counter_bad + st.counter_nothing),
                           "traffic": ctraffic,
                           "traffic_GBps": round(ctraffic / (c_ms / 1e3) / 1e9, 1) if ctraffic and c_ms > 0 else None},
        "stages_ms": {"ms_walk": round(max(r[1] for r in rows) * 1e3, 2),
                      "merge": round(max(r[2] for r in rows) * 1e3, 2),
                      "ms_walk_kernel": round(max(r[3] for r in rows), 2),
                      "counter_kernel": round(st.counter_kernel_ms, 2),
                      "note": "per step; N > 1: max over ranks of each rank's stage wall time"},
        "hbm_peak_gib": round(max(r[6] for r in rows) / 2**30, 2),
    }
    if world > 1:
        out["per_rank"] = [{"step_ms": round(r[0] / args.steps * 1e3, 2), "walk_ms": round(r[1] * 1e3, 2),
                            "merge_ms": round(r[2] * 1e3, 2), "walk_kernel_ms": round(r[3], 2),
                            "heads": int(r[4]), "chars": int(r[5]), "hbm_peak_gib": round(r[6] / 2**30, 2)}
                           for r in rows]
    if rank == 0 and not args.no_check:
        try:
            out["parity"] = parity_check(eng, args, rle)
        except Exception as e:  # reported, never fatal for the GPU number
            out["parity"] = {"error": str(e)[-400:]}
    if world > n_devices:
        out["rehearsal"] = f"{world} ranks on {n_devices} device(s): not a {world}-GPU measurement"
    if grp is not None:
        out["per_rank_devices"] = [int(r.device) for r in group_rows[-1]] if group_rows else None
        if group_rows:
            out["n_gpus"] = len(set(out["per_rank_devices"]))
        grp.close()
    else:
        eng.close()
    if rank == 0 and world == 1 and not args.no_e2e:
        try:
            out["e2e"] = e2e_leg(args, rle)
        except Exception as e:  # reported, never fatal for the GPU number
            out["e2e"] = {"error": str(e)[-400:]}
    if rank == 0 and not args.no_cpu:
        try:
            out["cpu_baseline"] = cpu_baseline(args.ref_len, args.cpu_copies, args.p, args.seed, rle=rle,
                                               full_copies=args.copies)
        except Exception as e:  # reported, never fatal for the GPU number
            out["cpu_baseline"] = {"error": str(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
