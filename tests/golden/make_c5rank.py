"""Config-5 rank-share golden (run in the build container; needs the oracle).

BASELINE.json config 5 is a 100 MB reference + 200 copies @1 % SNP, plain
BWT, on 8 GPUs.  At W = 8 rank 0 owns the leading empty document and copies
1-25 (cmsbwt.dist.shard_range(200, 8, 0)), about 265 M heads: the merge state
one rank holds at config 5.  This script writes exactly that collection with
the product's counter-based generator (synth.h via oracle/_build/gen_synth:
L = 1e8, 25 copies, p = 0.01, seed 5 -- copies 1..25 of the 200-copy set are
the same bytes) and runs the oracle on it with plain output (FN:1631-1694).

Writes golden.json["c5rank"]: headNumber / keys / Rank / counter totals and
sha256 + size of the `.bwt`.  Oracle time ~1 h on one core; RSS is reported.
"""
import hashlib
import json
import os
import resource
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib  # noqa: E402

ARGS = [100_000_000, 25, 0.01, 5]


def sha(p):
    h = hashlib.sha256()
    with open(p, "rb") as f:
        for blk in iter(lambda: f.read(1 << 24), b""):
            h.update(blk)
    return h.hexdigest()


def main():
    L, C, p, seed = ARGS
    with tempfile.TemporaryDirectory(dir=os.environ.get("C5R_TMP")) as td:
        pre = os.path.join(td, "c5r")
        subprocess.run([oracle_lib.GEN, str(L), str(C), str(p), str(seed), pre], check=True,
                       stdout=subprocess.DEVNULL)
        t0 = time.time()
        rc, st, tt = oracle_lib.run(pre + ".ref.fa", pre + ".coll.fa", pre + "_p", rle=False)
        assert rc == 0, rc
        t1 = time.time()
        out = {"args": ARGS, "generator": "synth.h (tools/gen_synth)", "headNumber": st["heads"],
               "keys": st["keys"], "Rank": st["rank"], "counterBad": st["bad"], "counterGood": st["good"],
               "counterDoNothing": st["nothing"], "positions": st["positions"],
               "bwt_bytes": os.path.getsize(pre + "_p.bwt"), "bwt_sha256": sha(pre + "_p.bwt"),
               "oracle_seconds_plain": round(t1 - t0, 1), "oracle_stage_seconds": [round(x, 1) for x in tt],
               "oracle_max_rss_gib": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20, 2),
               "note": "rank 0's share of config 5 at W = 8 (leading empty document + copies 1-25); "
                       "oracle-derived (parity unpinned beyond the oracle)"}
    gp = os.path.join(HERE, "golden.json")
    g = json.load(open(gp))
    g["c5rank"] = out
    json.dump(g, open(gp, "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
