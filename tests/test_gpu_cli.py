"""GPU: the drop-in boundary — the `cmsbwt` process (main.cpp:85-132 + FN:1788-1797).

The CLI is run as a subprocess on list files, exactly as a user of the
reference runs `cmsbwt`: outputs (.rl_bwt / .bwt, .counterSmallerThanHead_true
on the small path) are compared with the golden sha256 / the oracle's files,
the .log with the reference's keys in the reference's order (SURVEY.md App. C,
FN:161-309, FN:1094-1627), and exit codes with main.cpp's (1 on I/O errors).
"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import cases

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "cms-bwt_amd", "build", "cmsbwt")
GOLD = os.path.join(ROOT, "tests", "golden")

# FN:161-309 (initialize_reference), then the large path FN:1094-1627
KEYS_LARGE = ["About to read ref", "n = ", "Reference (size = ", "ftello(infile): ", "sn: ",
              "Augmenting reference done in ", "Computing SA done in ", "\tComputing ISA...",
              "Computing ISA done in ", "Computing LCP and PLCP done in ", "Computing RMQ...",
              "Computing RMQ done in ", "Computing BWT...", "Computing BWT done in ", "Finished pre-processing",
              "Preprocessing done in ", "File is in memory", "_x.len: ", "_sx.len: ",
              "About to start main parsing loop...", "Finished parsing file of length: ", "phrasesSet.size(): ",
              "headNumber: ", "ndoc: ", "docBoundaries.size(): ", "Time to compute matching statistics: ",
              "Going to compute ranks for positions", "Rank: ", "libsais_int ran in ", "First rankToHead: ",
              "Last rankToHead: ", "Done computing ranks for positions in ", "currentSum: ",
              "Going to compute counterSmallerThanHead for positions", "counterBad: ", "counterGood: ",
              "counterDoNothing: ", "Done computing counterSmallerThanHead for positions in ",
              "Inverted data in bucketsForExpandedBWT"]
# the small path (FN:312-936) prints uniqueHeadNumber and capOfBufferSuffixes
# instead of phrasesSet.size() and Rank
KEYS_SMALL = [k for k in KEYS_LARGE if k not in ("phrasesSet.size(): ", "Rank: ")]
KEYS_SMALL.insert(KEYS_SMALL.index("ndoc: "), "uniqueHeadNumber: ")
KEYS_SMALL.insert(KEYS_SMALL.index("counterBad: "), "capOfBufferSuffixes = ")


def run_cli(args, cwd=None, env=None):
    e = dict(os.environ, **env) if env else None
    return subprocess.run([CLI] + args, capture_output=True, text=True, cwd=cwd, timeout=300, env=e)


def parse_log(path, keys):
    """Values after each key; asserts every key appears, in the given order."""
    text = open(path).read()
    vals, at = {}, 0
    for k in keys:
        i = text.find(k, at)
        assert i >= 0, f"log key {k!r} missing (or out of order) in {path}:\n{text}"
        j = i + len(k)
        e = text.find("\n", j)
        vals[k] = text[j:e if e >= 0 else len(text)]
        at = j
    return vals


def num(v):
    return int(v.split()[0])


def sha(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 24), b""):
            h.update(blk)
    return h.hexdigest()


def _gen_np():
    sys.path.insert(0, GOLD)
    import gen_np
    return gen_np


def _first_last_rank_to_head(dump, oracle):
    """FN:1468-1477: rankToHead[headToRank[i+1]] = i; First/Last print
    rankToHead[0] and rankToHead[H-1]."""
    h2r = oracle.load_dump(dump, "head2rank").astype(np.int64)
    H = len(h2r) - 1
    r2h = np.empty(H, dtype=np.int64)
    r2h[h2r[1:]] = np.arange(H)
    return int(r2h[0]), int(r2h[H - 1])


def test_cli_config1_both_formats_and_log(built, oracle, tmp_path):
    """Config 1 (1 MB ref + 10 copies @0.1 %, App. B run c1): `cmsbwt -r` and
    `cmsbwt` write the golden .rl_bwt / .bwt; the .log holds every key of the
    large path with the reference's recorded headNumber and the oracle's
    counts."""
    g = json.load(open(os.path.join(GOLD, "golden.json")))["c1"]
    pre = str(tmp_path / "c1")
    _gen_np().gen(1_000_000, 10, 0.001, 11, pre)
    dump = str(tmp_path / "dump")
    rc, ost, _ = oracle.run(pre + ".ref.fa", pre + ".coll.fa", str(tmp_path / "o"), rle=True, dump_dir=dump)
    assert rc == 0
    r = run_cli(["-r", "-o", pre + "_r", pre + ".list"])
    assert r.returncode == 0, r.stdout + r.stderr
    assert "==== Time elapsed:" in r.stdout and "Output format: RLE" in r.stdout
    assert sha(pre + "_r.rl_bwt") == g["rl_bwt_sha256"]
    v = parse_log(pre + "_r.log", KEYS_LARGE)
    coll = open(pre + ".coll.fa", "rb").read()
    docs, sn = cases.py_read_docs(coll)
    assert num(v["n = "]) == os.path.getsize(pre + ".ref.fa")
    assert v["Reference (size = "].startswith("1000000)")
    assert num(v["ftello(infile): "]) == len(coll) == num(v["sn: "]) == num(v["_sx.len: "])
    assert num(v["_x.len: "]) == 1000123  # 121 + 2 augmentation bytes
    assert num(v["Finished parsing file of length: "]) == sn
    assert num(v["headNumber: "]) == g["headNumber"] == ost["heads"] == num(v["currentSum: "])
    assert num(v["Rank: "]) == g["Rank"] == ost["rank"]
    assert num(v["ndoc: "]) == num(v["docBoundaries.size(): "]) == len(docs) + 1 == ost["D"]
    assert num(v["phrasesSet.size(): "]) == ost["positions"]
    assert (num(v["counterBad: "]), num(v["counterGood: "]), num(v["counterDoNothing: "])) == \
        (ost["bad"], ost["good"], ost["nothing"])
    assert (num(v["First rankToHead: "]), num(v["Last rankToHead: "])) == _first_last_rank_to_head(dump, oracle)
    # plain .bwt, default output basename = the list file name (main.cpp:79)
    r = run_cli([pre + ".list"])
    assert r.returncode == 0, r.stdout + r.stderr
    assert os.path.getsize(pre + ".list.bwt") == g["bwt_bytes"]
    assert sha(pre + ".list.bwt") == g["bwt_sha256"]
    assert os.path.exists(pre + ".list.log")


@pytest.mark.parametrize("env", [{"CMSBWT_OVERLAP_UPLOAD": "0"}, {"CMSBWT_HOST_READER": "1"}],
                         ids=["upload_after_index", "host_reader"])
def test_cli_ingest_paths_golden(built, tmp_path, env):
    """`cmsbwt_run` streams the collection into HBM while the reference index
    is built (default); the upload after the index (CMSBWT_OVERLAP_UPLOAD=0)
    and the host getline reader (FN:1138-1147) give the same golden .rl_bwt
    and headNumber on config 1."""
    g = json.load(open(os.path.join(GOLD, "golden.json")))["c1"]
    pre = str(tmp_path / "c1")
    _gen_np().gen(1_000_000, 10, 0.001, 11, pre)
    r = run_cli(["-r", "-o", pre + "_r", pre + ".list"], env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert sha(pre + "_r.rl_bwt") == g["rl_bwt_sha256"]
    v = parse_log(pre + "_r.log", KEYS_LARGE)
    assert num(v["headNumber: "]) == g["headNumber"]


def test_cli_config2_golden(built, tmp_path):
    """Config 2 at full size (10 MB + 100 copies, App. B run t3) through the
    CLI: the reference's recorded headNumber, the oracle's counters and sha256."""
    g = json.load(open(os.path.join(GOLD, "golden.json")))
    pre = str(tmp_path / "t3")
    _gen_np().gen(10_000_000, 100, 0.001, 3, pre)
    r = run_cli(["-r", "-o", pre + "_o", pre + ".list"])
    assert r.returncode == 0, r.stdout + r.stderr
    assert sha(pre + "_o.rl_bwt") == g["t3"]["rl_bwt_sha256"]
    v = parse_log(pre + "_o.log", KEYS_LARGE)
    assert num(v["headNumber: "]) == g["survey"]["t3"]["headNumber"] == 10057656
    assert num(v["Rank: "]) == g["t3"]["Rank"]
    assert (num(v["counterBad: "]), num(v["counterGood: "]), num(v["counterDoNothing: "])) == \
        (g["t3"]["counterBad"], g["t3"]["counterGood"], g["t3"]["counterDoNothing"])
    assert num(v["ndoc: "]) == 102


@pytest.mark.parametrize("case", [c for c in cases.small_cases()
                                  if c[0] in ("copies_5k_1pct", "blank_lines_and_empty_docs", "prefix_cut")],
                         ids=lambda c: c[0])
@pytest.mark.parametrize("rle", [True, False], ids=["rl_bwt", "bwt"])
def test_cli_small_path_side_output(built, oracle, tmp_path, case, rle):
    """References below 1e6 symbols take the small path (FN:1792): the CLI also
    writes .counterSmallerThanHead_true (FN:919-924) and logs the small path's
    keys; -p is passed through (FN:223, FN:1258-1263)."""
    d, rp, cp, prefix = cases.materialise(tmp_path, case)
    rc, ost, _ = oracle.run(rp, cp, os.path.join(d, "oracle"), rle=rle, prefix=prefix)
    assert rc == 0
    args = (["-r"] if rle else []) + (["-p", str(prefix)] if prefix != cases.UINT64_MAX else [])
    r = run_cli(args + ["-b", "3", "-o", os.path.join(d, "gpu"), os.path.join(d, "list.txt")])
    assert r.returncode == 0, r.stdout + r.stderr
    ext = ".rl_bwt" if rle else ".bwt"
    assert open(os.path.join(d, "gpu" + ext), "rb").read() == open(os.path.join(d, "oracle" + ext), "rb").read()
    assert open(os.path.join(d, "gpu.counterSmallerThanHead_true"), "rb").read() == \
        open(os.path.join(d, "oracle.counterSmallerThanHead_true"), "rb").read()
    v = parse_log(os.path.join(d, "gpu.log"), KEYS_SMALL)
    assert num(v["headNumber: "]) == ost["heads"]
    assert num(v["uniqueHeadNumber: "]) == ost["keys"]
    _, sn = cases.py_read_docs(open(cp, "rb").read(), prefix)
    assert num(v["Finished parsing file of length: "]) == sn
    # FN:713-727 with -b 3: min(sn, 3 * 2^30 as unsigned int) / 20 + 1
    assert num(v["capOfBufferSuffixes = "]) == min(sn, 3 << 30) // 20 + 1


def test_cli_exit_codes_on_missing_inputs(built, tmp_path):
    """main.cpp:91-115 and FN:156-160 / FN:216-219 exit(1): a missing list
    file, an unreadable reference, a missing collection.  The reference's
    errors after the log redirect land in <base>.log (main.cpp:118-119)."""
    r = run_cli([str(tmp_path / "nope.list")])
    assert r.returncode == 1 and "Error opening file" in r.stderr
    case = cases.small_cases()[0]
    d, rp, cp, _ = cases.materialise(tmp_path, case)
    bad = os.path.join(d, "bad.list")
    open(bad, "w").write(os.path.join(d, "missing_ref.fa") + "\n" + cp + "\n")
    r = run_cli(["-r", "-o", os.path.join(d, "b1"), bad])
    assert r.returncode == 1
    assert "Error opening file of base sequence" in open(os.path.join(d, "b1.log")).read()
    open(bad, "w").write(rp + "\n" + os.path.join(d, "missing_coll.fa") + "\n")
    r = run_cli(["-r", "-o", os.path.join(d, "b2"), bad])
    assert r.returncode == 1
    assert "Error opening file of sequence (" in open(os.path.join(d, "b2.log")).read()
    # the engine stays a drop-in after an error: a good run in the same directory
    r = run_cli(["-r", "-o", os.path.join(d, "ok"), os.path.join(d, "list.txt")])
    assert r.returncode == 0 and os.path.getsize(os.path.join(d, "ok.rl_bwt")) > 0


def test_computeBWT_python_mirror(built, oracle, tmp_path):
    """cmsbwt.computeBWT (the Python mirror of FN:1788) writes the same files
    as the CLI and returns the statistics of the .log."""
    import cmsbwt
    case = cases.small_cases()[1]
    d, rp, cp, prefix = cases.materialise(tmp_path, case)
    rc, ost, _ = oracle.run(rp, cp, os.path.join(d, "oracle"), rle=True, prefix=prefix)
    assert rc == 0
    st = cmsbwt.computeBWT(cmsbwt.Args(filename=os.path.join(d, "list.txt"), outname=os.path.join(d, "py"),
                                       format=True), rp, cp)
    assert open(os.path.join(d, "py.rl_bwt"), "rb").read() == open(os.path.join(d, "oracle.rl_bwt"), "rb").read()
    assert (st.heads, st.keys, st.rank) == (ost["heads"], ost["keys"], ost["rank"])
    with pytest.raises(cmsbwt.CmsBwtError) as e:
        cmsbwt.computeBWT(cmsbwt.Args(outname=os.path.join(d, "py2")), os.path.join(d, "nope.fa"), cp)
    assert e.value.code == cmsbwt.CMSBWT_EIO
