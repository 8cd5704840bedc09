"""GPU: BASELINE config 5 at one rank's real share.

Config 5 is a 100 MB reference + 200 copies @1 % SNP, plain .bwt, on 8 GPUs.
At W = 8 rank 0 owns the leading empty document and copies 1-25
(cmsbwt.dist.shard_range(200, 8, 0)): ~265 M heads, the merge state one rank
holds at config 5.  The same collection (synth.h, seed 5; gen_synth writes
copies 1..25 of the 200-copy set) goes through
  * the position-sharded merge at W = 1 (dist_merge.hip through cmsbwt.dist),
  * the sharded merge at W = 2 (gloo, both ranks on the test GPU, byte-range
    ingest of the FASTA file), and
  * the drop-in `cmsbwt -n 2` (in-process ranks, PEER transport),
and each plain .bwt must equal the oracle's (golden c5rank: sha256 and size,
headNumber, keys, Rank, the three counter totals; tests/golden/make_c5rank.py).
FN:1387-1694 (merge and plain writer) at a head count 1/8 of config 5's
2.1e9 (FN:1436-1456's int32 limits are lifted to uint32 here).
"""
import hashlib
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "cms-bwt_amd", "build")


def _sha(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 24), b""):
            h.update(blk)
    return h.hexdigest()


@pytest.fixture(scope="module")
def c5rank(tmp_path_factory):
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))["c5rank"]
    L, C, p, seed = g["args"]
    d = tmp_path_factory.mktemp("c5rank")
    pre = str(d / "c5r")
    subprocess.run([os.path.join(BUILD, "gen_synth"), str(L), str(C), str(p), str(seed), pre], check=True,
                   stdout=subprocess.DEVNULL, timeout=300)
    return pre, g


def _check_stats(st, g):
    assert st["heads"] == g["headNumber"]
    assert st["keys"] == g["keys"]
    assert st["rank"] == g["Rank"]
    assert (st["counter_bad"], st["counter_good"], st["counter_nothing"]) == \
        (g["counterBad"], g["counterGood"], g["counterDoNothing"])


def _check_bwt(path, g):
    assert os.path.getsize(path) == g["bwt_bytes"]
    assert _sha(path) == g["bwt_sha256"]


def test_c5rank_sharded_world1(engine, c5rank, tmp_path):
    import cmsbwt.dist as cdist
    pre, g = c5rank
    engine.initialize_reference(pre + ".ref.fa")
    engine.load_collection_file(pre + ".coll.fa")
    cdist.sharded_step(engine, "cuda:0", rle=False, xfer=cdist.Transport("cuda:0", 1, 0))
    st = engine.stats()
    _check_stats(st.as_dict(), g)
    out = str(tmp_path / "w1")
    engine.write_output(out, rle=False)
    _check_bwt(out + ".bwt", g)
    print(json.dumps({"c5rank_w1": {"heads": st.heads, "hbm_peak_gib": round(st.device_peak_bytes / 2**30, 2),
                                    "walk_s": round(st.t_ms_walk_s, 3), "merge_s": round(st.t_merge_s, 3)}}))


def test_c5rank_sharded_world2_gloo(c5rank, tmp_path):
    from test_multirank import spawn
    pre, g = c5rank
    work = str(tmp_path)
    out = str(tmp_path / "w2")
    json.dump({"ref": pre + ".ref.fa", "coll": pre + ".coll.fa", "rle": False, "out": out},
              open(os.path.join(work, "cfg.json"), "w"))
    spawn("gpu_sharded_files", 2, work, timeout=900)
    _check_stats(json.load(open(os.path.join(work, "stats.json"))), g)
    _check_bwt(out + ".bwt", g)


def test_c5rank_cli_two_ranks(c5rank, tmp_path):
    pre, g = c5rank
    lst = str(tmp_path / "c5r.list")
    open(lst, "w").write(f"{pre}.ref.fa\n{pre}.coll.fa\n")
    out = str(tmp_path / "n2")
    r = subprocess.run([os.path.join(BUILD, "cmsbwt"), "-n", "2", "-v", "-o", out, lst], capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    _check_bwt(out + ".bwt", g)
    log = open(out + ".log").read()
    assert f"headNumber: {g['headNumber']}" in log
    peaks = [ln for ln in log.splitlines() if ln.startswith("rank ")]
    print("\n".join(peaks))
