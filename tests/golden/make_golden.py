"""Regenerate tests/golden/ (run in the build container; needs the oracle).

* golden.json "survey": counts recorded in SURVEY.md (App. B runs, numpy
  generator of gen_np.py) from a survey-container build of the reference
  linked against a stand-in libsais -- the oracle reproduces them, but they do
  not pin parity (parity unpinned).
* golden.json "c1"/"t2": oracle outputs on those inputs (sha256 of .rl_bwt,
  run/symbol counts), used by the GPU tests as golden vectors.
* small/<case>/: tiny inputs with expected .rl_bwt / .bwt bytes.  These are
  ORACLE-DERIVED (the reference cannot be built here: its libsais submodule is
  empty); byte parity with the reference itself is unpinned for them.
* golden.json "provenance": which entries are reference-recorded and which
  are oracle-derived (kept across regenerations).
"""
import hashlib
import json
import os
import shutil
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
import cases  # noqa: E402
import gen_np  # noqa: E402
import oracle_lib  # noqa: E402

SURVEY = {  # SURVEY.md §6 / App. A-1 / App. B, reference binary runs
    "c1": {"args": [1_000_000, 10, 0.001, 11, 0], "headNumber": 87853},
    "t2": {"args": [1_000_000, 3, 0.001, 2, 60], "rl_symbols": 3001340, "bwt_bytes": 3000004},
    "t3": {"args": [10_000_000, 100, 0.001, 3, 0], "headNumber": 10057656},
    "t4": {"args": [10_000_000, 1000, 0.001, 4, 0], "headNumber": 100530836, "Rank": 54531265,
           "rl_runs": 135580980, "rl_bytes": 1220228820},
}
SMALL = ["copies_5k_1pct", "blank_lines_and_empty_docs", "headerless_multiline", "prefix_cut",
         "identical_copies", "tiny_docs"]


def sha(p):
    return hashlib.sha256(open(p, "rb").read()).hexdigest()


PROVENANCE_NOTE = "see golden.json 'provenance': only 'survey' is recorded from the reference itself"


def main():
    prev = json.load(open(os.path.join(HERE, "golden.json")))
    out = {"survey": SURVEY, "provenance": prev.get("provenance", {"note": PROVENANCE_NOTE})}
    with tempfile.TemporaryDirectory() as td:
        for key in ("c1", "t2"):
            L, C, p, seed, w = SURVEY[key]["args"]
            pre = os.path.join(td, key)
            gen_np.gen(L, C, p, seed, pre, w)
            rc, st, _ = oracle_lib.run(pre + ".ref.fa", pre + ".coll.fa", pre + "_r", rle=True)
            assert rc == 0
            rc2, _, _ = oracle_lib.run(pre + ".ref.fa", pre + ".coll.fa", pre + "_p", rle=False)
            assert rc2 == 0
            import numpy as np
            a = np.fromfile(pre + "_r.rl_bwt", dtype=np.uint8).reshape(-1, 9)
            sym = int(a[:, :8].copy().view("<u8").sum())
            out[key] = {"headNumber": st["heads"], "keys": st["keys"], "Rank": st["rank"],
                        "rl_runs": len(a), "rl_symbols": sym, "rl_bwt_sha256": sha(pre + "_r.rl_bwt"),
                        "bwt_bytes": os.path.getsize(pre + "_p.bwt"), "bwt_sha256": sha(pre + "_p.bwt")}
    sd = os.path.join(HERE, "small")
    shutil.rmtree(sd, ignore_errors=True)
    for case in cases.small_cases():
        if case[0] not in SMALL:
            continue
        d, rp, cp, prefix = cases.materialise(sd, case)
        for rle, ext in ((True, ".rl_bwt"), (False, ".bwt")):
            rc, _, _ = oracle_lib.run(rp, cp, os.path.join(d, "expected"), rle=rle, prefix=prefix)
            assert rc == 0
        for f in os.listdir(d):
            if f.endswith(".log") or f.endswith("_true") or f == "list.txt":
                os.remove(os.path.join(d, f))
        with open(os.path.join(d, "prefix.txt"), "w") as f:
            f.write(str(prefix))
    json.dump(out, open(os.path.join(HERE, "golden.json"), "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
