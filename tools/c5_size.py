"""Size BASELINE config 5 (100 MB reference + 200 copies @1 % SNP, plain) on
one GPU: the MS walk alone (cmsbwt_ms_walk, FN:1151-1385) over
  * the 8 document shards a W = 8 run would own (25 copies each), and
  * the whole 200 copies (20 GB of text in HBM),
reporting heads, walk time and the HBM high-water mark of each.  Prints one
JSON line per run and a summary."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cms-bwt_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref-len", type=int, default=100_000_000)
    ap.add_argument("--copies", type=int, default=200)
    ap.add_argument("--p", type=float, default=0.01)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--full", type=int, default=1, help="also walk all copies in one context")
    args = ap.parse_args()
    import cmsbwt
    from bench import synth_reference
    from cmsbwt.dist import shard_range
    ref = synth_reference(args.ref_len, args.seed)
    res = {"ref_len": args.ref_len, "copies": args.copies, "p": args.p, "seed": args.seed, "shards": []}
    eng = cmsbwt.Engine(0)
    t0 = time.perf_counter()
    eng.load_reference_bytes(ref)
    res["index_s"] = round(time.perf_counter() - t0, 2)
    for r in range(args.world):
        c0, c1 = shard_range(args.copies, args.world, r)
        eng.load_synth(args.seed, 1 + c0, c1 - c0, args.p, leading_empty_doc=(r == 0))
        t0 = time.perf_counter()
        eng.ms_walk()
        dt = time.perf_counter() - t0
        st = eng.stats()
        row = {"rank": r, "copies": c1 - c0, "heads": st.heads, "chars": st.chars, "walk_s": round(dt, 3),
               "walk_kernel_ms": round(st.ms_walk_kernel_ms, 1), "hbm_peak_gib": round(st.device_peak_bytes / 2**30, 2)}
        res["shards"].append(row)
        print(json.dumps(row), flush=True)
    res["heads_total_from_shards"] = sum(r["heads"] for r in res["shards"])
    eng.close()
    if args.full:
        eng = cmsbwt.Engine(0)
        eng.load_reference_bytes(ref)
        eng.load_synth(args.seed, 1, args.copies, args.p, leading_empty_doc=True)
        t0 = time.perf_counter()
        eng.ms_walk()
        dt = time.perf_counter() - t0
        st = eng.stats()
        res["full"] = {"heads": st.heads, "chars": st.chars, "walk_s": round(dt, 3),
                       "walk_kernel_ms": round(st.ms_walk_kernel_ms, 1),
                       "hbm_peak_gib": round(st.device_peak_bytes / 2**30, 2)}
        print(json.dumps({"full": res["full"]}), flush=True)
        eng.close()
    h = res.get("full", {}).get("heads", res["heads_total_from_shards"])
    res["heads_over_2_31"] = round(h / 2**31, 4)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
