"""CPU: the C-ABI library loads and exports every symbol of include/cmsbwt.h;
host-side logic (collection reader, suffix array) checked without a GPU."""
import os
import re

import numpy as np
import pytest

import cases

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol(built):
    import cmsbwt
    lib = cmsbwt.load_library()
    hdr = open(os.path.join(ROOT, "include", "cmsbwt.h")).read()
    declared = set(re.findall(r"\b(cmsbwt_[a-z_0-9]+)\s*\(", hdr))
    assert declared == set(cmsbwt.EXPORTED)
    for name in declared:
        assert hasattr(lib, name), name


def test_ctx_create_fails_cleanly_without_device(built):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import cmsbwt
    with pytest.raises(cmsbwt.CmsBwtError) as e:
        cmsbwt.Engine(0)
    assert e.value.code == cmsbwt.CMSBWT_EDEVICE


def test_cli_exists_and_prints_help(built):
    import subprocess
    r = subprocess.run([os.path.join(ROOT, "cms-bwt_amd", "build", "cmsbwt"), "-h"], capture_output=True, text=True)
    assert r.returncode == 255 and "Usage:" in r.stdout and "-r" in r.stdout


def test_cli_argument_and_list_file_exit_codes(built, tmp_path):
    """main.cpp:27-115, before any device work: -h, an unknown option and a
    wrong argument count exit(-1) (255); a missing list file, an empty first
    line and an empty (or blank) second line exit(1)."""
    import subprocess
    cli = os.path.join(ROOT, "cms-bwt_amd", "build", "cmsbwt")

    def run(*a):
        return subprocess.run([cli, *a], capture_output=True, text=True, timeout=60)
    assert run("-h").returncode == 255
    r = run("-z", "x.list")
    assert r.returncode == 255 and "Unknown option" in r.stdout
    r = run()
    assert r.returncode == 255 and "Invalid number of arguments" in r.stdout
    assert run("a.list", "b.list").returncode == 255
    r = run(str(tmp_path / "missing.list"))
    assert r.returncode == 1 and "Error opening file" in r.stderr
    for body, msg in ((b"\nb.fa\n", "first line"), (b"a.fa\n\n", "second line"), (b"a.fa\n  \t\n", "second line"),
                      (b"a.fa\n", "second line")):
        p = tmp_path / "l.list"
        p.write_bytes(body)
        r = run("-r", str(p))
        assert r.returncode == 1 and msg in r.stderr, (body, r.stderr)
    # echo of the command line and parameters (main.cpp:31-34, 74-80)
    p.write_bytes(b"\nb\n")
    r = run("-p", "123", "-b", "4", "-o", "base", str(p))
    assert "==== Command line:" in r.stdout and "Prefix length: 123" in r.stdout
    assert "Buffer size: 4 GB" in r.stdout and "Output basename: base" in r.stdout and "FULL" in r.stdout


# Reader quirks, each restated from the reference line that causes it.  The
# committed small goldens are oracle outputs (parity with the reference itself
# is unpinned for them); these are the line-by-line cross-checks.
READER_QUIRKS = [
    # FN:1138 `while (getline(...).good())`: a last line without '\n' sets eof,
    # good() is false and the line is dropped
    ("unterminated_last_line_dropped", b">a\nACGT\nGG", [b"", b"ACGT"]),
    # FN:1139 `line.empty() || line[0] == '>'` ends a document: a leading
    # header closes an empty first document (FN:1140 appends the separator)
    ("leading_header_empty_first_doc", b">a\nAC\n", [b"", b"AC"]),
    # FN:1139 blank lines end documents like headers; consecutive ones give
    # empty documents
    ("blank_lines_split", b"AC\n\n\nGT\n", [b"AC", b"", b"GT"]),
    # FN:1257-1266 `else if (!line.empty())` concatenates lines: headerless
    # multi-line input is one document, closed as the tail (FN:1269-1275)
    ("headerless_multiline_one_doc", b"AC\nGT\nTT\n", [b"ACGTTT"]),
    # FN:1269 the tail document only exists when content is non-empty
    ("no_tail_after_header", b"AC\n>b\n", [b"AC"]),
    # '\r' is data: getline splits on '\n' only
    ("crlf_kept", b">a\r\nAC\r\n", [b"", b"AC\r"]),
]


@pytest.mark.parametrize("name,body,docs", READER_QUIRKS, ids=[q[0] for q in READER_QUIRKS])
def test_reader_quirks_restated_from_reference_lines(built, tmp_path, name, body, docs):
    import cmsbwt
    assert cases.py_read_docs(body)[0] == docs
    p = str(tmp_path / "c.fa")
    open(p, "wb").write(body)
    assert cmsbwt.host_read_collection(p, cases.UINT64_MAX)[0] == docs


def test_reader_prefix_cut_arithmetic(built, tmp_path):
    """-p (FN:223 `_sn = min(file size, prefixLength)`, FN:1259-1262): the line at
    which charactersRead reaches _sn - 1 is cut to `size - (read - _sn) - 1`
    bytes and reading stops; the separator counted by a header is one of the
    _sn symbols (`-p 1003` -> 1002 symbols)."""
    import cmsbwt
    body = b">a\n" + b"A" * 10 + b"\n>b\n" + b"C" * 10 + b"\n"
    p = str(tmp_path / "c.fa")
    open(p, "wb").write(body)
    # read: '>a' -> 1, A*10 -> 11, '>b' -> 12, C*10 -> 22 >= sn-1 = 14 -> cut to 10 - (22-15) - 1 = 2
    want = [b"", b"A" * 10, b"CC"]
    assert cases.py_read_docs(body, 15)[0] == want
    assert cmsbwt.host_read_collection(p, 15)[0] == want


@pytest.mark.parametrize("case", cases.small_cases(), ids=lambda c: c[0])
def test_reader_matches_reference_semantics(built, tmp_path, case):
    import cmsbwt
    d, rp, cp, prefix = cases.materialise(tmp_path, case)
    docs, sn = cmsbwt.host_read_collection(cp, prefix)
    want, want_sn = cases.py_read_docs(case[2], prefix)
    assert docs == want and sn == want_sn


def _naive_sa(s: bytes):
    return np.array(sorted(range(len(s)), key=lambda i: s[i:]), dtype=np.int32)


@pytest.mark.parametrize("seed", range(6))
def test_suffix_array_sais(built, seed):
    import cmsbwt
    rng = np.random.default_rng(seed)
    for n, sigma in ((1, 4), (2, 2), (17, 1), (300, 2), (1000, 4), (2000, 256)):
        s = bytes(rng.integers(0, sigma, n).astype(np.uint8)) if sigma > 1 else b"A" * n
        assert np.array_equal(cmsbwt.host_suffix_array(s), _naive_sa(s))
    s = b"ACGT" * 300 + b"\x01\x00"
    assert np.array_equal(cmsbwt.host_suffix_array(s), _naive_sa(s))


@pytest.mark.parametrize("world", [1, 2, 3, 5, 8])
def test_shard_bounds_split_at_document_ends(built, tmp_path, world):
    """cmsbwt_host_shard_bounds (multi-GPU ingest): bounds are monotone, start
    at 0, end at the file size, and parsing each slice with the reference's
    reader semantics (cases.py_read_docs, FN:1138-1275) and concatenating in
    rank order gives the whole file's documents."""
    import cmsbwt
    rng = np.random.default_rng(world)
    bodies = [c[2] for c in cases.small_cases() if c[3] == cases.UINT64_MAX]
    bodies += [b"", b"ACGT", b">", b"\n\n\n", b">x\nACGT\n>y\n", b"AC\nGT\n\n\nTT\n>h\nAAA",
               b">" + b"h" * 5000 + b"\n" + b"ACGT" * 3000 + b"\n>" + b"g" * 7000]
    for i, body in enumerate(bodies):
        p = tmp_path / f"c{i}.fa"
        p.write_bytes(body)
        b = cmsbwt.host_shard_bounds(str(p), world)
        assert b[0] == 0 and b[-1] == len(body) and all(x <= y for x, y in zip(b, b[1:]))
        want, _ = cases.py_read_docs(body)
        got = []
        for k in range(world):
            got += cases.py_read_docs(body[b[k]:b[k + 1]])[0]
        assert got == want, (i, world, b)


def test_walk_alignment_memo_search_replica(tmp_path):
    """The alignment memo of the walk (ms_walk2.hip)
    finds, in one cooperative round, the first mismatch and the next one (or
    how far the bytes are clean) from per-thread differences and per-piece
    ballots; a host replica of that search equals brute force on 200 k random
    slots."""
    import shutil
    import subprocess
    src = os.path.join(ROOT, "tools", "memo_check.cpp")
    exe = str(tmp_path / "memo_check")
    subprocess.run([shutil.which("g++") or "g++", "-O2", "-o", exe, src], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("bad 0"), r.stdout[-500:]


def test_bench_refuses_rank_mismatch():
    """bench.py must not print a line whose n_gpus differs from the ranks that
    run: --gpus 2 under WORLD_SIZE=1 exits 2 before touching a GPU."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"], cwd=root, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "refusing" in json.loads(r.stdout.strip().splitlines()[-1])["error"]


def test_bench_refuses_shared_devices_cpu():
    """In-process --gpus N with fewer devices than ranks (none here), or
    torchrun ranks all put on device 0, exit 2 without the explicit rehearsal
    variable, before touching a GPU."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "CMSBWT_BENCH_REHEARSAL", "CMSBWT_BENCH_SAME_GPU")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"], cwd=root, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, r.stderr[-1000:]
    assert "share a device" in json.loads(r.stdout.strip().splitlines()[-1])["error"]
    env2 = dict(env, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", CMSBWT_BENCH_SAME_GPU="1")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"], cwd=root, env=env2,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, r.stderr[-1000:]
    assert "REHEARSAL" in json.loads(r.stdout.strip().splitlines()[-1])["error"]


def test_walk_built_without_vgpr_liverange_pass():
    """ms_walk2.o must be built with SIOptimizeVGPRLiveRange off: that backend
    pass miscompiles the walk (DESIGN.md §3.1 round 6,
    profiles/r06_memo_miscompile.txt)."""
    mk = open(os.path.join(ROOT, "Makefile")).read()
    assert "-amdgpu-opt-vgpr-liverange=false" in mk
    rule = mk[mk.index("$(OUT)/ms_walk2.o:"):]
    assert "$(W2FLAGS)" in rule.splitlines()[1]
