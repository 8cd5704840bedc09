"""GPU parity: every stage of the HIP path equals the CPU oracle, bit for bit.

Stages (oracle dump name -> reference file:line):
  h_start/h_pos/h_len/h_smaller/h_lchar  heads of the MS walk   FN:1151-1212
  h_isa/h_tonext/h_nexthead              j-scan                 FN:1359-1385
  bucket                                  per-position counts    FN:1162-1185
  rank2head / head2rank                   ranks, libsais_int     FN:1432-1459
  bwtheads                                BWTheads               FN:1468-1472
  counters                                counterSmallerThanHead FN:1523-1603
  .rl_bwt / .bwt bytes                    writers                FN:1631-1777
"""
import os

import numpy as np
import pytest

import cases

pytestmark = pytest.mark.gpu

STAGES = ["h_start", "h_pos", "h_len", "h_smaller", "h_lchar", "h_isa", "h_tonext", "h_nexthead",
          "bucket", "rank2head", "head2rank", "bwtheads", "counters"]


def _compare(engine, oracle, tmp_path, case, chunk=None, rle=True, env=None):
    d, rp, cp, prefix = cases.materialise(tmp_path, case)
    dump = os.path.join(d, "dump")
    rc, ost, _ = oracle.run(rp, cp, os.path.join(d, "oracle"), rle=rle, prefix=prefix, dump_dir=dump)
    assert rc == 0
    env = dict(env or {})
    if chunk:
        env["CMSBWT_CHUNK"] = str(chunk)
    os.environ.update(env)
    try:
        engine.initialize_reference(rp)
        engine.load_collection_file(cp, prefix)
        engine.ms_walk()
        engine.merge(rle)
    finally:
        for k in env:
            os.environ.pop(k, None)
    for s in STAGES:
        got, want = engine.array(s), oracle.load_dump(dump, s)
        assert got.shape == want.shape, f"{case[0]}: {s} shape {got.shape} vs {want.shape}"
        if not np.array_equal(got, want):
            bad = np.nonzero(got != want)[0]
            raise AssertionError(f"{case[0]}: stage {s} differs at {len(bad)} entries, first {bad[:5]} "
                                 f"got {got[bad[:5]]} want {want[bad[:5]]}")
    st = engine.stats()
    assert st.heads == ost["heads"] and st.keys == ost["keys"] and st.rank == ost["rank"]
    assert (st.counter_bad, st.counter_good, st.counter_nothing) == (ost["bad"], ost["good"], ost["nothing"])
    out = os.path.join(d, "gpu")
    engine.write_output(out, rle)
    ext = ".rl_bwt" if rle else ".bwt"
    with open(out + ext, "rb") as f1, open(os.path.join(d, "oracle") + ext, "rb") as f2:
        assert f1.read() == f2.read(), f"{case[0]}: {ext} bytes differ"
    if st.n < 1_000_000:
        with open(out + ".counterSmallerThanHead_true", "rb") as f1, \
                open(os.path.join(d, "oracle.counterSmallerThanHead_true"), "rb") as f2:
            assert f1.read() == f2.read()
    return st


@pytest.mark.parametrize("case", cases.small_cases(), ids=lambda c: c[0])
def test_small_cases_rle(engine, oracle, tmp_path, case):
    _compare(engine, oracle, tmp_path, case, rle=True)


@pytest.mark.parametrize("case", cases.small_cases(), ids=lambda c: c[0])
def test_small_cases_generic_walk(engine, oracle, tmp_path, case):
    """The generic walk instance on every small case: CMSBWT_PFX_GENERIC=1
    sends DNA references there too (the specialised instance serves only DNA
    with every table).  Both instances run the alignment memo (DESIGN.md
    §3.1); the generic one needed a register barrier at a memo hit, without
    which the -O2/-O3 build recorded pos = i + K + 1 for the hit's head on
    every case here (tools/memo_repro.py) -- FN:45-88, FN:1151-1212."""
    _compare(engine, oracle, tmp_path, case, rle=True, env={"CMSBWT_PFX_GENERIC": "1"})


@pytest.mark.parametrize("case", cases.small_cases()[:6], ids=lambda c: c[0])
def test_small_cases_plain_bwt(engine, oracle, tmp_path, case):
    _compare(engine, oracle, tmp_path, case, rle=False)


@pytest.mark.parametrize("env", [{"CMSBWT_WR_SEGBUF": "0"}, {"CMSBWT_WR_UNFUSED": "1"}],
                         ids=["segments_recomputed", "unfused_writer"])
@pytest.mark.parametrize("rle", [True, False], ids=["rl_bwt", "bwt"])
@pytest.mark.parametrize("case", cases.small_cases()[:5], ids=lambda c: c[0])
def test_writer_variants(engine, oracle, tmp_path, case, rle, env):
    """The tile writer (default) keeps each element's segments between its
    two passes (16-byte packed form, elem_writer.h segs_pack); recomputing
    them in the second pass, and the element-scan writer of rounds 2-4,
    give the same bytes."""
    _compare(engine, oracle, tmp_path, case, rle=rle, env=env)


@pytest.mark.parametrize("rle", [True, False], ids=["rl_bwt", "bwt"])
@pytest.mark.parametrize("case", cases.small_cases()[:5], ids=lambda c: c[0])
def test_writer_two_scans(engine, oracle, tmp_path, case, rle):
    """Writer offsets (FN:1631-1777) by two 64-bit scans, the path taken
    when run and symbol totals do not fit one packed scan."""
    _compare(engine, oracle, tmp_path, case, rle=rle, env={"CMSBWT_WR_TWO_SCANS": "1"})


@pytest.mark.parametrize("rle", [True, False], ids=["rl_bwt", "bwt"])
@pytest.mark.parametrize("case", cases.ambiguity_cases(), ids=lambda c: c[0])
def test_comparator_ambiguity_replay(engine, oracle, tmp_path, case, rle):
    """match.h:27-33 is not a strict weak order on these inputs (bytes >= 0x80,
    signed compare at FN:55 vs unsigned suffix order): positions with
    ambiguous items get their std::map layout replayed on the host, and
    queries into them or ambiguous queries are answered there (map_replay.h);
    every stage equals the oracle, which runs the reference's std::map."""
    st = _compare(engine, oracle, tmp_path, case, rle=rle)
    assert st.order_violations > 0 and st.host_queries > 0


@pytest.mark.parametrize("case", cases.small_cases()[:6], ids=lambda c: c[0])
def test_forced_map_replay(engine, oracle, tmp_path, case):
    """CMSBWT_FORCE_REPLAY=1 rebuilds every position's items by the std::map
    replay and answers every counter query on the host: the replay machinery
    itself reproduces the oracle on consistent inputs."""
    st = _compare(engine, oracle, tmp_path, case, env={"CMSBWT_FORCE_REPLAY": "1"})
    # every query into a position with heads went to the host
    assert st.host_queries >= st.counter_bad + st.counter_good


@pytest.mark.parametrize("chunk", [64, 257, 1000])
@pytest.mark.parametrize("case", cases.small_cases()[:4], ids=lambda c: c[0])
def test_chunk_restarts(engine, oracle, tmp_path, case, chunk):
    """Tiny chunks force many restart points inside documents."""
    _compare(engine, oracle, tmp_path, case, chunk=chunk)


@pytest.mark.parametrize("geom", [{"CMSBWT_COUNTER_WIN": "1", "CMSBWT_WINPOS": "7"},
                                  {"CMSBWT_COUNTER_WIN": "1", "CMSBWT_WINPOS": "64", "CMSBWT_WINSLOTS": "16"},
                                  {"CMSBWT_COUNTER_WIN": "1", "CMSBWT_WINSLOTS": "1"},
                                  {"CMSBWT_FORCE_CHECK": "1", "CMSBWT_WINPOS": "33"}],
                         ids=["tiny_windows", "small_lds", "global_atomics", "checked_queries"])
@pytest.mark.parametrize("case", cases.small_cases()[:5], ids=lambda c: c[0])
def test_counter_window_geometry(engine, oracle, tmp_path, case, geom):
    """Slot-budget kernel (k_counter_win): tiny windows stress the crossing
    lists; slot caps below a position's slot count force its global-atomic
    fallback; checked queries always run here."""
    _compare(engine, oracle, tmp_path, case, env=geom)


@pytest.mark.parametrize("case", cases.small_cases()[:4], ids=lambda c: c[0])
def test_grouping_three_sorts(engine, oracle, tmp_path, case):
    """Grouping (FN:1387-1416) by three LSD sorts (the path for fields wider
    than one 64-bit key) gives the oracle's items, ranks and runs."""
    _compare(engine, oracle, tmp_path, case, env={"CMSBWT_GROUP3": "1"})


@pytest.mark.parametrize("env", [{"CMSBWT_TGTWIN": "7"}, {"CMSBWT_TGTWIN": "1"}, {"CMSBWT_TGTWIN": "64"},
                                 {"CMSBWT_TGTWIN": "200"}, {"CMSBWT_COUNTER_WIN": "1"},
                                 {"CMSBWT_XW_SORT": "1"}, {"CMSBWT_XW_SORT": "1", "CMSBWT_TGTWIN": "7"}],
                         ids=["tiny_windows", "one_target_windows", "one_wave_windows", "ragged_windows",
                              "slot_windows_kernel", "sorted_crossing_lists", "sorted_crossing_lists_tiny"])
@pytest.mark.parametrize("case", cases.small_cases()[:6], ids=lambda c: c[0])
def test_counter_target_major(engine, oracle, tmp_path, case, env):
    """counterSmallerThanHead (FN:1523-1603) target-major with per-lane
    accumulators: tiny windows stress the crossing lists (placed by distance,
    k_xw_*; one-target windows make sources deeper than kXwMaxDepth, which
    take the sort), windows of one wave or not a multiple of 64 targets leave
    waves idle or partly filled; the sorted crossing lists and the slot-budget
    kernel (k_counter_win) stay selectable."""
    _compare(engine, oracle, tmp_path, case, env=env)


@pytest.mark.parametrize("env", [{"CMSBWT_GROUP64": "1"}, {"CMSBWT_GROUP_SMALL": "1"},
                                 {"CMSBWT_GROUP_SMALL": "0"}],
                         ids=["one_key_sort", "long_segments", "all_segments_radix"])
@pytest.mark.parametrize("case", cases.small_cases()[:6], ids=lambda c: c[0])
def test_grouping_position_first(engine, oracle, tmp_path, case, env):
    """Grouping (FN:1387-1416) by a position radix sort plus per-position
    segment sorts (default), by one sort of the composite key, and with every
    segment longer than the per-thread limit (radix-sorted subset)."""
    _compare(engine, oracle, tmp_path, case, env=env)


@pytest.mark.parametrize("env", [{"CMSBWT_DBL_SMALL": "2"}, {"CMSBWT_DBL_SMALL": "1000000"},
                                 {"CMSBWT_DBL_LEADERS": "1"}, {"CMSBWT_DBL_LEADERS": "1", "CMSBWT_DBL_SMALL": "2"},
                                 {"CMSBWT_NHR_SORT": "1"}, {"CMSBWT_UNRES_BYTES": "1"}],
                         ids=["radix_groups", "member_ranks", "leader_sorts", "leader_radix", "nhr_item_sorts",
                              "unresolved_byte_flags"])
@pytest.mark.parametrize("case", cases.small_cases()[:4], ids=lambda c: c[0])
def test_doubling_group_paths(engine, oracle, tmp_path, case, env):
    """Head-string suffix sort: groups above CMSBWT_DBL_SMALL members go through
    the radix path, smaller ones are ranked per member (default) or sorted by
    their leader thread; all give the oracle's SA.  Next-head ranks (FN:1480-
    1494) ranked per slot (default) or sorted per item.  Unresolved members
    flagged in bit 31 of their sa entry (default) or in a byte per position."""
    _compare(engine, oracle, tmp_path, case, env=env)


@pytest.mark.parametrize("env", [{"CMSBWT_COUNTER_OVERLAP": "1"}, {"CMSBWT_COUNTER_OVERLAP": "1", "CMSBWT_EQ_CAP": "1"},
                                 {"CMSBWT_COUNTER_STATS": "2"}],
                         ids=["counter_beside_ranks", "equal_key_overflow", "pair_shape_stats"])
@pytest.mark.parametrize("case", cases.small_cases()[:6], ids=lambda c: c[0])
def test_counter_stream_paths(engine, oracle, tmp_path, case, env):
    """counterSmallerThanHead (FN:1523-1603) on the side stream beside the
    ranks and the suffix sort: the equal-key queries (FN:1537-1589, the only
    ones that read next-head ranks) are listed and answered after the ranks
    (k_counter_eq); an overflowing list (capacity 1) runs the counter again
    with the ranks.  The pair-shape statistics pass leaves the output alone."""
    _compare(engine, oracle, tmp_path, case, env=env)


@pytest.mark.parametrize("geom", [{"CMSBWT_RUN_BIN_SHIFT": "3", "CMSBWT_GRP_RUNS": "0"},
                                  {"CMSBWT_RUN_BIN_SHIFT": "5", "CMSBWT_RUN_BIN_GLOBAL": "1", "CMSBWT_GRP_RUNS": "0"},
                                  {"CMSBWT_RUN_BIN_GLOBAL": "1", "CMSBWT_GRP_RUNS": "0"}],
                         ids=["bins8_lds", "bins32_global", "bins8192_global"])
@pytest.mark.parametrize("case", cases.small_cases(), ids=lambda c: c[0])
def test_run_bucket_bins(engine, oracle, tmp_path, case, geom):
    """Run buckets (FN:1162-1171, 1203) through position bins: many small bins
    (runs crossing bin edges, endpoints at n) and the global-counter path used
    above kRunBinLdsMax bins give the oracle's bucket array and output
    (CMSBWT_GRP_RUNS=0: the grouping leaves the run ends to this path)."""
    _compare(engine, oracle, tmp_path, case, env=geom)


@pytest.mark.parametrize("env", [{"CMSBWT_PFX_GENERIC": "1"}, {"CMSBWT_KMER_BITS": "12"}, {"CMSBWT_PFX": "0"},
                                 {"CMSBWT_PFX_GENERIC": "1", "CMSBWT_CHUNK": "100"}, {"CMSBWT_PFX_PAIR": "0"}],
                         ids=["generic_symbol_map", "short_tables", "no_tables", "generic_tiny_chunks",
                              "unpaired_prefetch"])
@pytest.mark.parametrize("case", cases.small_cases()[:6] + cases.small_cases()[-3:], ids=lambda c: c[0])
def test_walk_table_paths(engine, oracle, tmp_path, case, env):
    """The walk's ways to the next character give the same heads: answer
    entries with the ACGT decode or the generic byte map, short tables (more
    heads at depth >= K: child table and binary searches), no tables at all
    (binary searches and adjustInterval scans only), many restarts, and the
    probe prefetch without the paired level-K table (CMSBWT_PFX_PAIR=0)."""
    _compare(engine, oracle, tmp_path, case, env=env)


@pytest.mark.parametrize("env", [{"CMSBWT_ROCPRIM_SCAN": "1"}, {"CMSBWT_ROCPRIM_SELECT": "1"},
                                 {"CMSBWT_W2_STATS": "1", "CMSBWT_DBL_STATS": "1", "CMSBWT_COUNTER_STATS": "1",
                                  "CMSBWT_TIMING": "1"},
                                 {"CMSBWT_HOST_INDEX": "1"}],
                         ids=["rocprim_scans", "rocprim_select", "instrumented", "host_index"])
@pytest.mark.parametrize("case", cases.small_cases()[:4] + cases.small_cases()[-1:], ids=lambda c: c[0])
def test_fallback_and_instrumented_paths(engine, oracle, tmp_path, case, env):
    """rocPRIM scans / compaction instead of the tile kernels, the statistics
    builds (the walk's STATS instantiation, doubling/counter counters, index
    timing) and the host-built index all leave every stage bit-exact."""
    _compare(engine, oracle, tmp_path, case, env=env)


@pytest.mark.parametrize("case", cases.large_cases(), ids=lambda c: c[0])
def test_large_reference_path(engine, oracle, tmp_path, case):
    _compare(engine, oracle, tmp_path, case, rle=True)


def test_config1_golden(engine, tmp_path):
    """SURVEY.md config 1 (1 MB ref + 10 copies @0.1%, numpy generator of App. B,
    seed 11): the reference recorded headNumber 87,853; the committed sha256 of
    the oracle's .rl_bwt is the golden vector."""
    import json
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import gen_np
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))["c1"]
    pre = str(tmp_path / "c1")
    gen_np.gen(1_000_000, 10, 0.001, 11, pre)
    engine.initialize_reference(pre + ".ref.fa")
    engine.load_collection_file(pre + ".coll.fa")
    engine.step(rle=True)
    import hashlib
    st = engine.stats()
    assert st.heads == g["headNumber"] == 87853
    assert hashlib.sha256(engine.runs_bytes()).hexdigest() == g["rl_bwt_sha256"]


def test_bench_workload_generated_in_hbm_matches_files(engine, oracle, tmp_path):
    """bench.py's data path: the collection generated in HBM (synth.hip) and the
    reference from bench.synth_reference give the same .rl_bwt as the oracle on
    the FASTA files written by tools/gen_synth."""
    import subprocess
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(__file__)))
    import bench
    L, C, p, seed = 300_000, 5, 0.002, 4
    pre = str(tmp_path / "s")
    subprocess.run([oracle.GEN, str(L), str(C), str(p), str(seed), pre], check=True)
    assert oracle.run(pre + ".ref.fa", pre + ".coll.fa", pre + "_o", rle=True)[0] == 0
    engine.load_reference_bytes(bench.synth_reference(L, seed))
    engine.load_synth(seed, 1, C, p, leading_empty_doc=True)
    engine.step(rle=True)
    assert engine.runs_bytes() == open(pre + "_o.rl_bwt", "rb").read()


def test_bench_workload_full_size_golden(engine):
    """bench.py's headline step at full size (synth.h: 10 MB ref + 1000 copies
    @0.1 %, generated in HBM) equals the oracle's .rl_bwt on the same workload
    written as FASTA by gen_synth (golden synth_c3: sha256, heads, Rank and
    counter statistics; the oracle took 1675 s on one core)."""
    import hashlib
    import json
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(__file__)))
    import bench
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))["synth_c3"]
    L, C, p, seed = g["args"]
    engine.load_reference_bytes(bench.synth_reference(L, seed))
    engine.load_synth(seed, 1, C, p, leading_empty_doc=True)
    engine.step(rle=True)
    st = engine.stats()
    assert (st.heads, st.keys, st.rank, st.runs) == (g["headNumber"], g["keys"], g["Rank"], g["rl_runs"])
    assert (st.counter_bad, st.counter_good, st.counter_nothing) == \
        (g["counterBad"], g["counterGood"], g["counterDoNothing"])
    assert hashlib.sha256(engine.runs_bytes()).hexdigest() == g["rl_bwt_sha256"]


def test_repeated_steps_identical(engine, tmp_path):
    """The caching allocator reuses buffers across steps: three steps on the
    same inputs must give identical runs (and match across rle/plain reruns)."""
    case = cases.small_cases()[1]
    d, rp, cp, prefix = cases.materialise(tmp_path, case)
    engine.initialize_reference(rp)
    engine.load_collection_file(cp, prefix)
    outs = []
    for rle in (True, False, True, True):
        engine.step(rle=rle)
        outs.append(engine.runs_bytes())
    assert outs[0] == outs[2] == outs[3]


def test_config2_full_size_golden(engine, tmp_path):
    """SURVEY.md config 2 at full size (10 MB ref + 100 copies @0.1%, 1 GB,
    numpy generator seed 3): headNumber equals the reference's recorded
    10,057,656 and the .rl_bwt equals the oracle's (sha256 committed)."""
    import hashlib
    import json
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import gen_np
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))
    pre = str(tmp_path / "t3")
    gen_np.gen(10_000_000, 100, 0.001, 3, pre)
    engine.initialize_reference(pre + ".ref.fa")
    engine.load_collection_file(pre + ".coll.fa")
    engine.step(rle=True)
    st = engine.stats()
    assert st.heads == g["survey"]["t3"]["headNumber"] == 10057656
    assert (st.counter_bad, st.counter_good, st.counter_nothing) == \
        (g["t3"]["counterBad"], g["t3"]["counterGood"], g["t3"]["counterDoNothing"])
    assert hashlib.sha256(engine.runs_bytes()).hexdigest() == g["t3"]["rl_bwt_sha256"]


def test_config3_full_size_golden(engine):
    """The headline workload at full size: 10 MB ref + 1000 copies @0.1 %
    (10 GB, numpy generator seed 4, SURVEY App. B run t4).  headNumber, Rank
    and run count equal the reference's recorded values; the .rl_bwt equals the
    oracle's (sha256 committed; the oracle took 1125 s on one core)."""
    import hashlib
    import json
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import gen_np
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))
    ref, text, off = gen_np.gen_arrays(10_000_000, 1000, 0.001, 4)
    engine.load_reference_bytes(ref)
    engine.load_collection_array(text, off)
    del text
    engine.step(rle=True)
    st = engine.stats()
    assert st.heads == g["survey"]["t4"]["headNumber"] == 100530836
    assert st.rank == g["survey"]["t4"]["Rank"]
    assert st.runs == g["survey"]["t4"]["rl_runs"] == 135580980
    assert (st.counter_bad, st.counter_good, st.counter_nothing) == \
        (g["t4"]["counterBad"], g["t4"]["counterGood"], g["t4"]["counterDoNothing"])
    assert hashlib.sha256(engine.runs_bytes()).hexdigest() == g["t4"]["rl_bwt_sha256"]


def _sha_file(path):
    import hashlib
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 24), b""):
            h.update(blk)
    return h.hexdigest()


def test_config5_proxy_golden(engine, tmp_path):
    """BASELINE config 5's shape (100 MB reference, 1 % SNP, plain .bwt) on the
    proxy SURVEY.md §8(a) prescribes, since the reference path cannot run the
    full 200 copies: 100 MB ref + 4 copies @1 % (numpy generator seed 5).
    Head/key/rank counts, counter statistics and the sha256 of both the plain
    .bwt and the .rl_bwt equal the oracle's (tests/golden/make_c5proxy.py)."""
    import json
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import gen_np
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))["c5p"]
    L, C, p, seed, _ = g["args"]
    ref, text, off = gen_np.gen_arrays(L, C, p, seed)
    engine.load_reference_bytes(ref)
    engine.load_collection_array(text, off)
    del text
    engine.step(rle=False)
    st = engine.stats()
    assert st.heads == g["headNumber"]
    assert st.rank == g["Rank"]
    assert (st.counter_bad, st.counter_good, st.counter_nothing) == \
        (g["counterBad"], g["counterGood"], g["counterDoNothing"])
    out = str(tmp_path / "c5p")
    engine.write_output(out, rle=False)
    assert os.path.getsize(out + ".bwt") == g["bwt_bytes"]
    assert _sha_file(out + ".bwt") == g["bwt_sha256"]
    engine.step(rle=True)
    assert engine.stats().runs == g["rl_runs"]
    import hashlib
    assert hashlib.sha256(engine.runs_bytes()).hexdigest() == g["rl_bwt_sha256"]


@pytest.mark.parametrize("threads,chunk_mb", [("3", "1"), ("8", "32")])
def test_writer_streams_both_formats(engine, tmp_path, threads, chunk_mb):
    """Output files through the pinned writer (device .bwt expansion, pwrite
    threads): 1 MiB chunks over 3 writers split the 10 MB .bwt and the 7.6 MB
    .rl_bwt of config 1 into many chunks; both equal the golden sha256."""
    import hashlib
    import json
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import gen_np
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))["c1"]
    pre = str(tmp_path / "c1")
    gen_np.gen(1_000_000, 10, 0.001, 11, pre)
    env = {"CMSBWT_WRITE_THREADS": threads, "CMSBWT_READ_CHUNK_MB": chunk_mb}
    os.environ.update(env)
    try:
        engine.initialize_reference(pre + ".ref.fa")
        engine.load_collection_file(pre + ".coll.fa")
        for rle, ext, key in ((True, ".rl_bwt", "rl_bwt_sha256"), (False, ".bwt", "bwt_sha256")):
            engine.step(rle=rle)
            with open(pre + "_gpu" + ext, "wb") as f:  # an older, longer output is overwritten and cut
                f.write(b"\xff" * 25_000_000)
            engine.write_output(pre + "_gpu", rle)
            assert hashlib.sha256(open(pre + "_gpu" + ext, "rb").read()).hexdigest() == g[key], ext
    finally:
        for k in env:
            os.environ.pop(k, None)
    assert os.path.getsize(pre + "_gpu.bwt") == g["bwt_bytes"]


@pytest.mark.parametrize("case", cases.large_cases(), ids=lambda c: c[0])
def test_large_reference_run_bins_beyond_lds(engine, oracle, tmp_path, case):
    """1 M reference with 32-position bins: 31k bins exceed kRunBinLdsMax, so
    the bin counters take the global path on their own."""
    _compare(engine, oracle, tmp_path, case, rle=True, env={"CMSBWT_RUN_BIN_SHIFT": "5"})


@pytest.mark.parametrize("host_reader", [False, True], ids=["device_reader", "host_reader"])
@pytest.mark.parametrize("case", cases.no_document_cases(), ids=lambda c: c[0])
def test_collection_without_documents(engine, tmp_path, case, host_reader):
    """Zero documents: the walk yields no heads (no chunk is read), and the merge
    refuses with CMSBWT_EINPUT where the reference is undefined (FN:1359-1385),
    as the oracle does (tests/test_oracle.py)."""
    import cmsbwt
    d, rp, cp, prefix = cases.materialise(tmp_path, case)
    engine.initialize_reference(rp)
    # a -p prefix above the file size keeps the host reader
    engine.load_collection_file(cp, (1 << 62) if host_reader else prefix)
    engine.ms_walk()
    st = engine.stats()
    assert (st.heads, st.ndocs) == (0, 0)
    assert not engine.array("diff").any() and not engine.array("hashead").any()
    with pytest.raises(cmsbwt.CmsBwtError) as ei:
        engine.merge(True)
    assert ei.value.code == cmsbwt.CMSBWT_EINPUT
    # the engine stays usable afterwards
    case2 = cases.small_cases()[0]
    d2, rp2, cp2, _ = cases.materialise(tmp_path, case2)
    engine.initialize_reference(rp2)
    engine.load_collection_file(cp2)
    engine.step(rle=True)
    assert engine.stats().heads > 0


@pytest.mark.parametrize("case", cases.small_cases(), ids=lambda c: c[0])
def test_small_cases_without_stage_copies(engine, oracle, tmp_path, case):
    """The production merge keeps no parity copies (CMSBWT_KEEP_STAGES=0, as
    bench.py and the CLI run it; the unresolved flags then stay in bit 31 of
    the sa entries, cleared before a head2rank copy).  The runs and the
    statistics equal the oracle's."""
    d, rp, cp, prefix = cases.materialise(tmp_path, case)
    rc, ost, _ = oracle.run(rp, cp, os.path.join(d, "oracle"), rle=True, prefix=prefix)
    assert rc == 0
    want = open(os.path.join(d, "oracle") + ".rl_bwt", "rb").read()
    old = os.environ.get("CMSBWT_KEEP_STAGES")
    os.environ["CMSBWT_KEEP_STAGES"] = "0"
    try:
        engine.initialize_reference(rp)
        engine.load_collection_file(cp, prefix)
        engine.ms_walk()
        engine.merge(True)
    finally:
        if old is None:
            del os.environ["CMSBWT_KEEP_STAGES"]
        else:
            os.environ["CMSBWT_KEEP_STAGES"] = old
    assert engine.runs_bytes() == want
    st = engine.stats()
    assert (st.heads, st.keys, st.rank) == (ost["heads"], ost["keys"], ost["rank"])
    assert (st.counter_bad, st.counter_good, st.counter_nothing) == (ost["bad"], ost["good"], ost["nothing"])
    h2r = engine.array("head2rank")  # (int32: a flag left in bit 31 would read negative)
    assert int(h2r.min()) >= 0
