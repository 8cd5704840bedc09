"""CPU: checks of the oracle before anything is compared against it.
Parity with the reference itself is UNPINNED: the reference
holds no fixtures and cannot be built here (empty libsais submodule).

1. Its plain .bwt equals a brute-force multi-string BWT (mathematical definition).
2. It reproduces the counts SURVEY.md recorded from a survey-container build
   of the reference linked against a stand-in libsais (config 1 headNumber
   87,853; the RLE-quirk symbol count 3,001,340 vs 3,000,004 plain bytes on
   t2), using the survey's numpy generator.  A consistency check, not a pin.
3. It matches the committed small golden files (regression)."""
import json
import os

import numpy as np
import pytest

import cases

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _decode(path):
    a = np.fromfile(path, dtype=np.uint8).reshape(-1, 9)
    return a[:, :8].copy().view("<u8").ravel(), a[:, 8].copy()


@pytest.mark.parametrize("case", cases.small_cases(), ids=lambda c: c[0])
def test_oracle_plain_bwt_is_the_multistring_bwt(oracle, tmp_path, case):
    d, rp, cp, prefix = cases.materialise(tmp_path, case)
    rc, st, _ = oracle.run(rp, cp, os.path.join(d, "o"), rle=False, prefix=prefix)
    assert rc == 0
    docs, _ = cases.py_read_docs(case[2], prefix)
    got = open(os.path.join(d, "o.bwt"), "rb").read()
    assert got == cases.brute_force_bwt(docs)
    assert st["D"] == len(docs) + 1


@pytest.mark.parametrize("case", cases.small_cases()[:5], ids=lambda c: c[0])
def test_oracle_rle_decodes_to_bwt_plus_quirk(oracle, tmp_path, case):
    """.rl_bwt differs from RLE(.bwt) only by the per-item remainder (App. A-1):
    it never has fewer symbols, and run chars alternate."""
    d, rp, cp, prefix = cases.materialise(tmp_path, case)
    assert oracle.run(rp, cp, os.path.join(d, "o"), rle=True, prefix=prefix)[0] == 0
    assert oracle.run(rp, cp, os.path.join(d, "o"), rle=False, prefix=prefix)[0] == 0
    lens, chars = _decode(os.path.join(d, "o.rl_bwt"))
    assert (lens > 0).all() and (chars[1:] != chars[:-1]).all()
    assert int(lens.sum()) >= os.path.getsize(os.path.join(d, "o.bwt"))


@pytest.mark.parametrize("case", cases.no_document_cases(), ids=lambda c: c[0])
def test_oracle_rejects_collection_without_documents(oracle, tmp_path, case):
    """Zero documents means zero heads, where FN:1359-1385 is undefined: the
    oracle refuses (rc 3, "reference UB") instead of reading V[-1]."""
    d, rp, cp, prefix = cases.materialise(tmp_path, case)
    assert cases.py_read_docs(case[2], prefix)[0] == []
    rc, st, _ = oracle.run(rp, cp, os.path.join(d, "o"), rle=True, prefix=prefix)
    assert rc == 3 and st["heads"] == 0


def _gen(tmp_path, key):
    import sys
    sys.path.insert(0, GOLD)
    import gen_np
    g = json.load(open(os.path.join(GOLD, "golden.json")))
    L, C, p, seed, w = g["survey"][key]["args"]
    pre = str(tmp_path / key)
    gen_np.gen(L, C, p, seed, pre, w)
    return g, pre


def test_oracle_reproduces_reference_config1(oracle, tmp_path):
    g, pre = _gen(tmp_path, "c1")
    rc, st, _ = oracle.run(pre + ".ref.fa", pre + ".coll.fa", pre + "_o", rle=True)
    assert rc == 0
    assert st["heads"] == g["survey"]["c1"]["headNumber"] == 87853
    import hashlib
    assert hashlib.sha256(open(pre + "_o.rl_bwt", "rb").read()).hexdigest() == g["c1"]["rl_bwt_sha256"]


def test_oracle_reproduces_reference_rle_quirk_t2(oracle, tmp_path):
    g, pre = _gen(tmp_path, "t2")
    assert oracle.run(pre + ".ref.fa", pre + ".coll.fa", pre + "_r", rle=True)[0] == 0
    assert oracle.run(pre + ".ref.fa", pre + ".coll.fa", pre + "_p", rle=False)[0] == 0
    lens, _ = _decode(pre + "_r.rl_bwt")
    assert int(lens.sum()) == g["survey"]["t2"]["rl_symbols"] == 3001340
    assert os.path.getsize(pre + "_p.bwt") == g["survey"]["t2"]["bwt_bytes"] == 3000004


@pytest.mark.parametrize("name", sorted(os.listdir(os.path.join(GOLD, "small"))))
def test_oracle_matches_committed_small_goldens(oracle, tmp_path, name):
    d = os.path.join(GOLD, "small", name)
    prefix = int(open(os.path.join(d, "prefix.txt")).read())
    out = str(tmp_path / "o")
    for rle, ext in ((True, ".rl_bwt"), (False, ".bwt")):
        assert oracle.run(os.path.join(d, "ref.fa"), os.path.join(d, "coll.fa"), out, rle=rle, prefix=prefix)[0] == 0
        assert open(out + ext, "rb").read() == open(os.path.join(d, "expected" + ext), "rb").read()


@pytest.mark.parametrize("case", cases.ambiguity_cases(), ids=lambda c: c[0])
def test_ambiguity_cases_break_the_map_order(oracle, tmp_path, case):
    """The crafted inputs of the std::map replay tests really break
    match.h:27-33's strict weak order: some position holds a smaller=true and
    a smaller=false head of the same length whose isaNext values are in the
    opposite order.  (The reference's output is then not the
    multi-string BWT: parity means the oracle's std::map layout, not the
    brute-force BWT.)"""
    d, rp, cp, prefix = cases.materialise(tmp_path, case)
    dump = os.path.join(d, "dump")
    rc, st, _ = oracle.run(rp, cp, os.path.join(d, "o"), rle=False, prefix=prefix, dump_dir=dump)
    assert rc == 0
    pos, ln = oracle.load_dump(dump, "h_pos").astype(np.int64), oracle.load_dump(dump, "h_len").astype(np.int64)
    sm, isa = oracle.load_dump(dump, "h_smaller"), oracle.load_dump(dump, "h_isa").astype(np.int64)
    key = (pos << 32) | ln
    tmax, fmin = {}, {}
    for k, s, i in zip(key.tolist(), sm.tolist(), isa.tolist()):
        if s:
            tmax[k] = max(tmax.get(k, -1), i)
        else:
            fmin[k] = min(fmin.get(k, 1 << 40), i)
    assert sum(1 for k in tmax if k in fmin and fmin[k] <= tmax[k]) > 0
