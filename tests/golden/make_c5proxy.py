"""Config-5 proxy golden (run in the build container; needs the oracle).

BASELINE.json config 5 is a 100 MB reference + 200 copies @1 % SNP, plain BWT.
SURVEY.md §8(a) "Config-5 risk": the reference path cannot run it (int32 head
ranks at FN:1436-1437/1456, ~200 GB of state), so its parity is pinned on a
scaled-down proxy with the same reference size, divergence and output mode:
100 MB reference + 4 copies @1 % (numpy generator of gen_np.py, seed 5).

Writes golden.json["c5p"]: oracle headNumber / keys / Rank, sha256 and size of
the plain `.bwt`, and sha256 / run count of the `.rl_bwt` of the same input.
"""
import hashlib
import json
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
import gen_np  # noqa: E402
import oracle_lib  # noqa: E402

ARGS = [100_000_000, 4, 0.01, 5, 0]


def sha(p):
    h = hashlib.sha256()
    with open(p, "rb") as f:
        for blk in iter(lambda: f.read(1 << 24), b""):
            h.update(blk)
    return h.hexdigest()


def main():
    L, C, p, seed, w = ARGS
    with tempfile.TemporaryDirectory(dir=os.environ.get("C5P_TMP")) as td:
        pre = os.path.join(td, "c5p")
        gen_np.gen(L, C, p, seed, pre, w)
        t0 = time.time()
        rc, st, tt = oracle_lib.run(pre + ".ref.fa", pre + ".coll.fa", pre + "_p", rle=False)
        assert rc == 0, rc
        t1 = time.time()
        rc2, st2, _ = oracle_lib.run(pre + ".ref.fa", pre + ".coll.fa", pre + "_r", rle=True)
        assert rc2 == 0, rc2
        runs = os.path.getsize(pre + "_r.rl_bwt") // 9
        out = {"args": ARGS, "headNumber": st["heads"], "keys": st["keys"], "Rank": st["rank"],
               "counterBad": st["bad"], "counterGood": st["good"], "counterDoNothing": st["nothing"],
               "bwt_bytes": os.path.getsize(pre + "_p.bwt"), "bwt_sha256": sha(pre + "_p.bwt"),
               "rl_runs": runs, "rl_bwt_sha256": sha(pre + "_r.rl_bwt"),
               "oracle_seconds_plain": round(t1 - t0, 1), "oracle_stage_seconds": [round(x, 1) for x in tt]}
    gp = os.path.join(HERE, "golden.json")
    g = json.load(open(gp))
    g["c5p"] = out
    json.dump(g, open(gp, "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
