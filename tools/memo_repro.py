"""Reproducer for the walk's alignment memo.

Runs the MS walk of the small parity cases through one library build
(CMSBWT_LIB, e.g. a CMSBWT_MEMO_GENERIC=1 / CMSBWT_MEMO_CHECK=1 build made with
`make lib OUT=exp/<v> XFLAGS=...`) in the generic walk instance
(CMSBWT_PFX_GENERIC=1 also sends DNA references there) and in the default
one, and compares the head records with the oracle's (FN:1151-1212).  For the
first differing head it prints the text and reference bytes around it.
Test infrastructure: uses the oracle as the checker.

  python tools/memo_repro.py [case-name ...]
"""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cms-bwt_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ.setdefault("CMSBWT_KEEP_STAGES", "1")

import numpy as np  # noqa: E402

import cases  # noqa: E402
import cmsbwt  # noqa: E402
import oracle_lib  # noqa: E402

HEAD = ["h_start", "h_pos", "h_len", "h_smaller"]


def run_case(eng, case, td, generic):
    d, rp, cp, prefix = cases.materialise(td, case)
    dump = os.path.join(d, "dump")
    if not os.path.exists(os.path.join(dump, "h_pos.u32")):
        rc, _, _ = oracle_lib.run(rp, cp, os.path.join(d, "oracle"), rle=True, prefix=prefix, dump_dir=dump)
        assert rc == 0
    if generic:
        os.environ["CMSBWT_PFX_GENERIC"] = "1"
    try:
        eng.initialize_reference(rp)
        eng.load_collection_file(cp, prefix)
        eng.ms_walk()
    finally:
        os.environ.pop("CMSBWT_PFX_GENERIC", None)
    got = {s: eng.array(s) for s in HEAD}
    want = {s: oracle_lib.load_dump(dump, s) for s in HEAD}
    tag = f"{case[0]:28s} {'generic' if generic else 'default'}"
    if all(got[s].shape == want[s].shape and np.array_equal(got[s], want[s]) for s in HEAD):
        print(f"{tag} ok ({len(want['h_pos'])} heads)", flush=True)
        return True
    # first differing head in document order
    n = min(len(got["h_pos"]), len(want["h_pos"]))
    k = next((j for j in range(n) if any(got[s][j] != want[s][j] for s in HEAD)), n)
    print(f"{tag} DIFF: {len(got['h_pos'])} heads vs {len(want['h_pos'])}; first at head {k}", flush=True)
    for j in range(max(0, k - 3), min(n, k + 4)):
        g = tuple(int(got[s][j]) for s in HEAD)
        w = tuple(int(want[s][j]) for s in HEAD)
        print(f"   head {j}: got (start,pos,len,smaller)={g} want={w}{'  <--' if g != w else ''}")
    return False


def main():
    names = set(sys.argv[1:])
    sel = [c for c in cases.small_cases() if not names or c[0] in names]
    print("library:", cmsbwt._LIB_PATH, flush=True)
    ok = True
    with tempfile.TemporaryDirectory() as td, cmsbwt.Engine(0) as eng:
        for c in sel:
            for generic in (True, False):
                ok &= run_case(eng, c, td, generic)
    print("ALL OK" if ok else "SOME DIFFER", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
