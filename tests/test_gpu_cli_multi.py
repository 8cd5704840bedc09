"""GPU: the drop-in's multi-GPU path -- `cmsbwt -n N` (SURVEY.md §8(b)
`n_gpus`; main.cpp:85-132 + FN:1788-1797 on N ranks in one process).

Ranks wrap over the devices, so on the one-GPU test box `-n 4` runs four
ranks (contexts, streams, caching allocators) on device 0 and the PEER
transport's pulls are device-local copies; on a node they are
hipMemcpyPeerAsync over xGMI.  Every output must equal the one-GPU /
oracle bytes, and the .log every value of the one-GPU run's log."""
import json
import os

import pytest

import cases
from test_gpu_cli import CLI, GOLD, KEYS_LARGE, KEYS_SMALL, _gen_np, num, parse_log, run_cli, sha

pytestmark = pytest.mark.gpu

TIMERS = ("done in", "ran in", "milliseconds", " ms")


def _values(path, keys):
    """Log values that do not depend on timing."""
    v = parse_log(path, keys)
    return {k: x for k, x in v.items() if not any(t in k + x for t in TIMERS)}


@pytest.mark.parametrize("n", [2, 4])
def test_cli_multi_config2_golden(built, tmp_path, n):
    """Config 2 (10 MB + 100 copies, 1 GB) with -n 2 / -n 4: each rank reads
    its byte range and the merge runs sharded by reference position; the
    .rl_bwt equals the golden t3 sha256 and the log the reference's counts."""
    g = json.load(open(os.path.join(GOLD, "golden.json")))
    pre = str(tmp_path / "t3")
    _gen_np().gen(10_000_000, 100, 0.001, 3, pre)
    r = run_cli(["-r", "-n", str(n), "-v", "-o", pre + "_o", pre + ".list"])
    assert r.returncode == 0, r.stdout + r.stderr
    assert sha(pre + "_o.rl_bwt") == g["t3"]["rl_bwt_sha256"]
    v = parse_log(pre + "_o.log", KEYS_LARGE)
    assert num(v["headNumber: "]) == g["survey"]["t3"]["headNumber"] == 10057656 == num(v["currentSum: "])
    assert num(v["Rank: "]) == g["t3"]["Rank"]
    assert (num(v["counterBad: "]), num(v["counterGood: "]), num(v["counterDoNothing: "])) == \
        (g["t3"]["counterBad"], g["t3"]["counterGood"], g["t3"]["counterDoNothing"])
    assert num(v["ndoc: "]) == 102
    log = open(pre + "_o.log").read()
    assert sum(f"rank {k} (device" in log for k in range(n)) == n


def test_cli_multi_config1_log_equals_one_gpu(built, tmp_path):
    """Config 1 with -n 3, both formats: the outputs equal the golden files and
    every non-timing value of the .log (phrasesSet.size, First/Last rankToHead,
    _sn, ...) equals the one-GPU run's."""
    g = json.load(open(os.path.join(GOLD, "golden.json")))["c1"]
    pre = str(tmp_path / "c1")
    _gen_np().gen(1_000_000, 10, 0.001, 11, pre)
    r1 = run_cli(["-r", "-o", pre + "_1", pre + ".list"])
    r3 = run_cli(["-r", "-n", "3", "-o", pre + "_3", pre + ".list"])
    assert r1.returncode == 0 and r3.returncode == 0, r3.stdout + r3.stderr
    assert sha(pre + "_3.rl_bwt") == sha(pre + "_1.rl_bwt") == g["rl_bwt_sha256"]
    assert _values(pre + "_3.log", KEYS_LARGE) == _values(pre + "_1.log", KEYS_LARGE)
    r = run_cli(["-n", "3", "-o", pre + "_3p", pre + ".list"])
    assert r.returncode == 0, r.stdout + r.stderr
    assert sha(pre + "_3p.bwt") == g["bwt_sha256"]


@pytest.mark.parametrize("env", [{"CMSBWT_DIST": "gather"}, {"CMSBWT_HOST_READER": "1"},
                                 {"CMSBWT_DM_FORCE_GATHER": "1"}],
                         ids=["gather", "host_reader", "ambiguity_fallback"])
def test_cli_multi_gather_paths(built, tmp_path, env):
    """The gather merge (every rank's heads to rank 0, one-GPU merge there)
    and the host reader's document split give the same golden bytes; so does
    the comparator-ambiguity fallback (sharded step, then the walk again and a
    gather step), forced by its test hook."""
    g = json.load(open(os.path.join(GOLD, "golden.json")))["c1"]
    pre = str(tmp_path / "c1")
    _gen_np().gen(1_000_000, 10, 0.001, 11, pre)
    r = run_cli(["-r", "-n", "2", "-o", pre + "_g", pre + ".list"], env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert sha(pre + "_g.rl_bwt") == g["rl_bwt_sha256"]
    assert num(parse_log(pre + "_g.log", KEYS_LARGE)["headNumber: "]) == g["headNumber"]


@pytest.mark.parametrize("n", [2, 3])
@pytest.mark.parametrize("case", [c for c in cases.small_cases()
                                  if c[0] in ("copies_5k_1pct", "blank_lines_and_empty_docs", "prefix_cut",
                                              "tiny_docs")],
                         ids=lambda c: c[0])
def test_cli_multi_small_path(built, oracle, tmp_path, case, n):
    """References below 1e6 symbols on N ranks: the heads are gathered on rank
    0 (the small path's .counterSmallerThanHead_true needs every counter); -p
    is read by the host reader and its documents split over the ranks."""
    d, rp, cp, prefix = cases.materialise(tmp_path, case)
    rc, ost, _ = oracle.run(rp, cp, os.path.join(d, "oracle"), rle=True, prefix=prefix)
    assert rc == 0
    args = ["-r"] + (["-p", str(prefix)] if prefix != cases.UINT64_MAX else [])
    r = run_cli(args + ["-n", str(n), "-o", os.path.join(d, "gpu"), os.path.join(d, "list.txt")])
    assert r.returncode == 0, r.stdout + r.stderr
    assert open(os.path.join(d, "gpu.rl_bwt"), "rb").read() == open(os.path.join(d, "oracle.rl_bwt"), "rb").read()
    assert open(os.path.join(d, "gpu.counterSmallerThanHead_true"), "rb").read() == \
        open(os.path.join(d, "oracle.counterSmallerThanHead_true"), "rb").read()
    v = parse_log(os.path.join(d, "gpu.log"), KEYS_SMALL)
    assert num(v["headNumber: "]) == ost["heads"]
    assert num(v["uniqueHeadNumber: "]) == ost["keys"]
    _, sn = cases.py_read_docs(open(cp, "rb").read(), prefix)
    assert num(v["Finished parsing file of length: "]) == sn


def test_cli_multi_more_ranks_than_documents(built, oracle, tmp_path):
    """-n 5 on a collection of 2 documents: three ranks own no bytes."""
    rng = cases._rng(31)
    ref = cases.rand_dna(rng, 3000)
    coll = cases.mutate(rng, ref, 0.01) + b"\n\n" + cases.mutate(rng, ref, 0.01) + b"\n"
    case = ("two_docs", cases.fasta([ref]), coll, cases.UINT64_MAX)
    d, rp, cp, prefix = cases.materialise(tmp_path, case)
    rc, ost, _ = oracle.run(rp, cp, os.path.join(d, "oracle"), rle=False, prefix=prefix)
    assert rc == 0
    r = run_cli(["-n", "5", "-o", os.path.join(d, "gpu"), os.path.join(d, "list.txt")])
    assert r.returncode == 0, r.stdout + r.stderr
    assert open(os.path.join(d, "gpu.bwt"), "rb").read() == open(os.path.join(d, "oracle.bwt"), "rb").read()


def test_cli_multi_errors(built, tmp_path):
    """A missing collection is still exit 1 with the reference's log line; a
    collection byte absent from the reference (reference UB) fails on its rank
    and the others leave cleanly; RCCL refuses ranks that share a GPU."""
    case = cases.small_cases()[0]
    d, rp, cp, _ = cases.materialise(tmp_path, case)
    bad = os.path.join(d, "bad.list")
    open(bad, "w").write(rp + "\n" + os.path.join(d, "missing_coll.fa") + "\n")
    r = run_cli(["-r", "-n", "2", "-o", os.path.join(d, "b1"), bad])
    assert r.returncode == 1
    assert "Error opening file of sequence (" in open(os.path.join(d, "b1.log")).read()
    ub = os.path.join(d, "ub.fa")
    open(ub, "wb").write(b">a\nACGT\n>b\nACGT\x90\x90\n>c\nACGT\n")  # a byte >= 0x80 absent from the reference
    open(bad, "w").write(rp + "\n" + ub + "\n")
    r = run_cli(["-r", "-n", "3", "-o", os.path.join(d, "b2"), bad])
    assert r.returncode == 2 + 3  # CMSBWT_EINPUT
    assert "does not occur in the reference" in open(os.path.join(d, "b2.log")).read()
    import torch
    if torch.cuda.device_count() == 1:
        r = run_cli(["-r", "-n", "2", "-t", "rccl", "-o", os.path.join(d, "b3"), os.path.join(d, "list.txt")])
        assert r.returncode == 2 + 2  # CMSBWT_EARG
        assert "distinct GPU" in open(os.path.join(d, "b3.log")).read()


def test_computeBWT_multi_python_mirror(built, oracle, tmp_path):
    """cmsbwt.computeBWT with Args(n_gpus=2) (the Python mirror of FN:1788)."""
    import cmsbwt
    case = cases.small_cases()[1]
    d, rp, cp, prefix = cases.materialise(tmp_path, case)
    rc, ost, _ = oracle.run(rp, cp, os.path.join(d, "oracle"), rle=True, prefix=prefix)
    assert rc == 0
    st = cmsbwt.computeBWT(cmsbwt.Args(outname=os.path.join(d, "py"), format=True, n_gpus=2,
                                       prefixLength=prefix), rp, cp)
    assert open(os.path.join(d, "py.rl_bwt"), "rb").read() == open(os.path.join(d, "oracle.rl_bwt"), "rb").read()
    assert (st.heads, st.keys) == (ost["heads"], ost["keys"])


def test_cli_multi_labels_past_2_31(built, tmp_path):
    """Config 1 with -n 2 and the sharded merge's group labels biased to
    straddle 2^31 (CMSBWT_DM_LABEL_BIAS; config 5's 2.12e9 heads sit at 0.986 x
    2^31): golden bytes, and First/Last rankToHead without the bias."""
    g = json.load(open(os.path.join(GOLD, "golden.json")))["c1"]
    pre = str(tmp_path / "c1")
    _gen_np().gen(1_000_000, 10, 0.001, 11, pre)
    r1 = run_cli(["-r", "-o", pre + "_1", pre + ".list"])
    r2 = run_cli(["-r", "-n", "2", "-o", pre + "_2", pre + ".list"],
                 env={"CMSBWT_DM_LABEL_BIAS": str(2**31 - g["headNumber"] // 2)})
    assert r1.returncode == 0 and r2.returncode == 0, r2.stdout + r2.stderr
    assert sha(pre + "_2.rl_bwt") == g["rl_bwt_sha256"]
    assert _values(pre + "_2.log", KEYS_LARGE) == _values(pre + "_1.log", KEYS_LARGE)


@pytest.mark.parametrize("backend", ["peer", "rccl"])
def test_cli_multi_injected_rank_failure(built, tmp_path, backend):
    """One rank fails after its walk (test hook CMSBWT_MULTI_FAIL_RANK) while
    the others enter the sharded merge's exchanges: the process ends with that
    rank's error code and log line, no crash and no hang.  With RCCL the
    failure aborts the communicators; the enqueue gate keeps every rank out of
    RCCL calls on them from then on.  RCCL needs one GPU per rank."""
    import torch
    if backend == "rccl" and torch.cuda.device_count() < 2:
        pytest.skip("RCCL needs two distinct GPUs")
    pre = str(tmp_path / "c1")
    _gen_np().gen(1_000_000, 10, 0.001, 11, pre)
    for fail_rank in ("1", "0"):
        r = run_cli(["-r", "-n", "2", "-t", backend, "-o", pre + "_f" + fail_rank, pre + ".list"],
                    env={"CMSBWT_MULTI_FAIL_RANK": fail_rank})
        assert r.returncode == 2 + 7, (r.returncode, r.stdout[-500:], r.stderr[-500:])  # CMSBWT_EINTERNAL
        assert f"rank {fail_rank}: injected failure" in open(pre + "_f" + fail_rank + ".log").read()
