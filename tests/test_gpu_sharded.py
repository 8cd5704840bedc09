"""GPU: the position-sharded merge (dist_merge.hip, cmsbwt.dist.sharded_step)
produces the oracle's .rl_bwt / .bwt bytes and statistics.

world == 1 runs every stage of the sharded pipeline in one process (identity
exchange); world 2 and 3 run as processes sharing the test GPU, exchanging over
gloo (host staging) exactly the collectives bench.py issues over RCCL."""
import json
import os

import pytest

import cases
from test_multirank import spawn

pytestmark = pytest.mark.gpu


def _oracle_files(oracle, tmp_path, case, rle):
    d, rp, cp, prefix = cases.materialise(tmp_path, case)
    rc, ost, _ = oracle.run(rp, cp, os.path.join(d, "oracle"), rle=rle, prefix=prefix)
    assert rc == 0
    want = open(os.path.join(d, "oracle") + (".rl_bwt" if rle else ".bwt"), "rb").read()
    return d, rp, cp, prefix, ost, want


def _expand(runs: bytes) -> bytes:
    import cmsbwt
    lens, chars = cmsbwt.decode_rl(runs)
    return b"".join(bytes([c]) * int(k) for k, c in zip(lens, chars))


@pytest.mark.parametrize("rle", [True, False], ids=["rl_bwt", "bwt"])
@pytest.mark.parametrize("case", cases.small_cases(), ids=lambda c: c[0])
def test_sharded_world1_matches_oracle(engine, oracle, tmp_path, case, rle):
    import cmsbwt.dist as cdist
    d, rp, cp, prefix, ost, want = _oracle_files(oracle, tmp_path, case, rle)
    engine.initialize_reference(rp)
    engine.load_collection_file(cp, prefix)
    cdist.sharded_step(engine, "cuda:0", rle=rle, xfer=cdist.Transport("cuda:0", 1, 0))
    runs = engine.runs_bytes()
    assert (runs if rle else _expand(runs)) == want
    st = engine.stats()
    assert (st.heads, st.keys, st.rank) == (ost["heads"], ost["keys"], ost["rank"])
    assert (st.counter_bad, st.counter_good, st.counter_nothing) == (ost["bad"], ost["good"], ost["nothing"])


@pytest.mark.parametrize("env", ["CMSBWT_GROUP3", "CMSBWT_GROUP64", "CMSBWT_WR_TWO_SCANS"])
@pytest.mark.parametrize("case", [c for c in cases.small_cases() if c[0] in ("copies_5k_1pct", "tiny_docs",
                                                                         "copies_20k_multiline")],
                         ids=lambda c: c[0])
def test_sharded_world1_composite_key_grouping(engine, oracle, tmp_path, case, env):
    """The grouping paths other than the position-first sort (taken when
    2 * bits(n) + bits(max len) > 64, e.g. config 5's 100 MB reference with
    long matches): the sharded merge then counts the run buckets of the
    received heads itself (k_dm_runs); bytes equal the oracle's."""
    import cmsbwt.dist as cdist
    d, rp, cp, prefix, ost, want = _oracle_files(oracle, tmp_path, case, True)
    os.environ[env] = "1"
    try:
        engine.initialize_reference(rp)
        engine.load_collection_file(cp, prefix)
        cdist.sharded_step(engine, "cuda:0", rle=True, xfer=cdist.Transport("cuda:0", 1, 0))
    finally:
        del os.environ[env]
    assert engine.runs_bytes() == want
    st = engine.stats()
    assert (st.heads, st.keys, st.rank) == (ost["heads"], ost["keys"], ost["rank"])


def _multi(oracle, tmp_path, case, world, rle, steps=1):
    d, rp, cp, prefix, ost, want = _oracle_files(oracle, tmp_path, case, rle)
    docs, _ = cases.py_read_docs(open(cp, "rb").read(), prefix)
    if len(docs) < world:
        pytest.skip("fewer documents than ranks")
    work = str(tmp_path)
    json.dump({"ref": rp, "docs": [x.hex() for x in docs], "rle": rle, "steps": steps},
              open(os.path.join(work, "cfg.json"), "w"))
    spawn("gpu_position_sharded", world, work)
    for it in range(steps):
        runs = open(os.path.join(work, f"runs{it}.bin"), "rb").read()
        assert (runs if rle else _expand(runs)) == want, f"step {it}"
    st = json.load(open(os.path.join(work, "stats.json")))
    assert (st["heads"], st["keys"], st["rank"]) == (ost["heads"], ost["keys"], ost["rank"])
    assert (st["counter_bad"], st["counter_good"], st["counter_nothing"]) == (ost["bad"], ost["good"], ost["nothing"])


MULTI = ["copies_5k_1pct", "copies_20k_multiline", "copies_3k_5pct", "identical_copies", "unrelated_random",
         "blank_lines_and_empty_docs", "tiny_docs", "prefix_cut"]


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("case", [c for c in cases.small_cases() if c[0] in MULTI], ids=lambda c: c[0])
def test_sharded_multi_rank_matches_oracle(oracle, tmp_path, case, world):
    _multi(oracle, tmp_path, case, world, rle=True)


@pytest.mark.parametrize("world", [1, 2])
@pytest.mark.parametrize("case", cases.ambiguity_cases()[:2], ids=lambda c: c[0])
def test_sharded_comparator_ambiguity_falls_back(engine, oracle, tmp_path, case, world):
    """Comparator ambiguity in the sharded merge: the step is
    redone as a gather step whose one-GPU merge replays std::map (world 1 in
    this process, world 2 over gloo); bytes equal the oracle's."""
    if world == 1:
        import cmsbwt.dist as cdist
        d, rp, cp, prefix, ost, want = _oracle_files(oracle, tmp_path, case, True)
        engine.initialize_reference(rp)
        engine.load_collection_file(cp, prefix)
        cdist.sharded_step(engine, "cuda:0", rle=True, xfer=cdist.Transport("cuda:0", 1, 0))
        assert engine.runs_bytes() == want
        st = engine.stats()
        assert (st.heads, st.keys, st.rank) == (ost["heads"], ost["keys"], ost["rank"])
        assert st.order_violations > 0
    else:
        _multi(oracle, tmp_path, case, world, rle=True)


def test_sharded_four_ranks_plain_bwt_repeated(oracle, tmp_path):
    case = ("copies_40k",) + cases.copies_case(7, 40000, 9, 0.004) + (cases.UINT64_MAX,)
    _multi(oracle, tmp_path, case, 4, rle=False, steps=2)


def test_sharded_world1_config3_golden(engine):
    """The headline workload at full size (10 MB ref + 1000 copies @0.1 %,
    10 GB, SURVEY App. B run t4) through every stage of the sharded merge:
    the .rl_bwt equals the oracle's (sha256 committed) and the reference's
    recorded headNumber / Rank / run count."""
    import hashlib
    import sys
    import cmsbwt.dist as cdist
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import gen_np
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))
    ref, text, off = gen_np.gen_arrays(10_000_000, 1000, 0.001, 4)
    engine.load_reference_bytes(ref)
    engine.load_collection_array(text, off)
    del text
    cdist.sharded_step(engine, "cuda:0", rle=True, xfer=cdist.Transport("cuda:0", 1, 0))
    st = engine.stats()
    assert st.heads == g["survey"]["t4"]["headNumber"]
    assert st.rank == g["survey"]["t4"]["Rank"]
    assert st.runs == g["survey"]["t4"]["rl_runs"]
    assert (st.counter_bad, st.counter_good, st.counter_nothing) == \
        (g["t4"]["counterBad"], g["t4"]["counterGood"], g["t4"]["counterDoNothing"])
    assert hashlib.sha256(engine.runs_bytes()).hexdigest() == g["t4"]["rl_bwt_sha256"]


def test_rank_without_documents(oracle, tmp_path):
    """More ranks than documents: the last rank owns none (its walk yields no
    heads, ms_walk returns without a chunk) and the position-sharded merge
    still gives the oracle's bytes."""
    rng = cases._rng(31)
    ref = cases.rand_dna(rng, 3000)
    coll = cases.mutate(rng, ref, 0.01) + b"\n\n" + cases.mutate(rng, ref, 0.01) + b"\n"  # blank line splits: 2 docs
    case = ("two_docs", cases.fasta([ref]), coll, cases.UINT64_MAX)
    d, rp, cp, prefix, ost, want = _oracle_files(oracle, tmp_path, case, True)
    docs, _ = cases.py_read_docs(coll, prefix)
    assert len(docs) == 2
    work = str(tmp_path)
    json.dump({"ref": rp, "docs": [x.hex() for x in docs], "rle": True, "steps": 1},
              open(os.path.join(work, "cfg.json"), "w"))
    spawn("gpu_position_sharded", 3, work)
    assert open(os.path.join(work, "runs0.bin"), "rb").read() == want
    st = json.load(open(os.path.join(work, "stats.json")))
    assert (st["heads"], st["keys"], st["rank"]) == (ost["heads"], ost["keys"], ost["rank"])


@pytest.mark.parametrize("case", [c for c in cases.small_cases() if c[0] in ("copies_5k_1pct", "tiny_docs")],
                         ids=lambda c: c[0])
def test_gather_step_device_tensors_rccl(oracle, tmp_path, case):
    """gather_step with device tensors over RCCL (one rank: RCCL allows one rank
    per GPU): the collectives and the root's copy are asynchronous on torch's
    stream, the engine reads on its own; two repeated steps equal the oracle."""
    d, rp, cp, prefix, ost, want = _oracle_files(oracle, tmp_path, case, True)
    docs, _ = cases.py_read_docs(open(cp, "rb").read(), prefix)
    work = str(tmp_path)
    json.dump({"ref": rp, "docs": [x.hex() for x in docs], "rle": True, "steps": 2},
              open(os.path.join(work, "cfg.json"), "w"))
    spawn("gpu_gather_device", 1, work)
    for it in range(2):
        assert open(os.path.join(work, f"runs{it}.bin"), "rb").read() == want, f"step {it}"


def test_sharded_eight_ranks_config2_files_golden(tmp_path):
    """BASELINE config 4's shape at config 2's size: 8 ranks (gloo, sharing the
    test GPU), each reading its byte range of the 1 GB FASTA collection
    (10 MB ref + 100 copies @0.1 %, App. B run t3) and running the
    position-sharded merge.  headNumber equals the reference's recorded
    10,057,656; the .rl_bwt equals the golden sha256."""
    import hashlib
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import gen_np
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))
    pre = str(tmp_path / "t3")
    gen_np.gen(10_000_000, 100, 0.001, 3, pre)
    work = str(tmp_path)
    json.dump({"ref": pre + ".ref.fa", "coll": pre + ".coll.fa", "rle": True},
              open(os.path.join(work, "cfg.json"), "w"))
    spawn("gpu_sharded_files", 8, work, timeout=600)
    st = json.load(open(os.path.join(work, "stats.json")))
    assert st["heads"] == g["survey"]["t3"]["headNumber"] == 10057656
    assert st["rank"] == g["t3"]["Rank"]
    assert (st["counter_bad"], st["counter_good"], st["counter_nothing"]) == \
        (g["t3"]["counterBad"], g["t3"]["counterGood"], g["t3"]["counterDoNothing"])
    assert hashlib.sha256(open(os.path.join(work, "runs0.bin"), "rb").read()).hexdigest() == g["t3"]["rl_bwt_sha256"]


def test_sharded_four_ranks_config5_proxy_plain_golden(tmp_path):
    """BASELINE config 5's shape (100 MB reference, 1 % SNP, plain .bwt) on the
    multi-GPU path: 4 ranks (gloo, sharing the test GPU) read their byte ranges
    of the c5p proxy's FASTA (4 copies, numpy generator seed 5) and run the
    position-sharded merge; rank 0 writes the plain .bwt, whose sha256 equals
    the oracle's (golden c5p), with the oracle's head / rank / counter counts."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import gen_np
    from test_gpu_parity import _sha_file
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))["c5p"]
    L, C, p, seed, _ = g["args"]
    pre = str(tmp_path / "c5p")
    gen_np.gen(L, C, p, seed, pre)
    work = str(tmp_path)
    out = str(tmp_path / "c5p_out")
    json.dump({"ref": pre + ".ref.fa", "coll": pre + ".coll.fa", "rle": False, "out": out},
              open(os.path.join(work, "cfg.json"), "w"))
    spawn("gpu_sharded_files", 4, work, timeout=600)
    st = json.load(open(os.path.join(work, "stats.json")))
    assert st["heads"] == g["headNumber"]
    assert st["rank"] == g["Rank"]
    assert (st["counter_bad"], st["counter_good"], st["counter_nothing"]) == \
        (g["counterBad"], g["counterGood"], g["counterDoNothing"])
    assert os.path.getsize(out + ".bwt") == g["bwt_bytes"]
    assert _sha_file(out + ".bwt") == g["bwt_sha256"]


# Config 5 has 2,118,018,850 heads (tools/c5_size.py): 0.986 x
# 2^31, so group labels of larger collections cross 2^31.  The sharded merge
# carries a label bias (CMSBWT_DM_LABEL_BIAS) through every label it moves,
# sorts and routes; biases just below 2^31 and near 2^32 make a small case's
# labels cross bit 31 / use all 32 bits, with the oracle's bytes expected.
LABEL_BIASES = [2**31 - 64, 2**32 - 2**20]


@pytest.mark.parametrize("bias", LABEL_BIASES, ids=["straddle_2_31", "near_2_32"])
@pytest.mark.parametrize("world", [1, 2])
def test_sharded_labels_past_2_31(engine, oracle, tmp_path, world, bias, monkeypatch):
    monkeypatch.setenv("CMSBWT_DM_LABEL_BIAS", str(bias))
    case = [c for c in cases.small_cases() if c[0] == "copies_5k_1pct"][0]
    if world == 1:
        import cmsbwt.dist as cdist
        d, rp, cp, prefix, ost, want = _oracle_files(oracle, tmp_path, case, True)
        assert ost["heads"] > 64
        engine.initialize_reference(rp)
        engine.load_collection_file(cp, prefix)
        cdist.sharded_step(engine, "cuda:0", rle=True, xfer=cdist.Transport("cuda:0", 1, 0))
        assert engine.runs_bytes() == want
        st = engine.stats()
        assert (st.heads, st.keys, st.rank) == (ost["heads"], ost["keys"], ost["rank"])
        assert (st.counter_bad, st.counter_good, st.counter_nothing) == (ost["bad"], ost["good"], ost["nothing"])
    else:
        _multi(oracle, tmp_path, case, world, rle=True)
