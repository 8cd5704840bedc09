"""GPU collection reader (coll_read.hip) against the host
reader, which restates the reference's getline loop (FN:1138-1275) and is
itself checked against a Python restatement in test_host.py.

Documents, separators, offsets, `sn` and the byte check must be identical on
every edge case: headers and blank lines, an unterminated last line, CRLF,
headerless input, lines and headers that straddle 16 KiB tiles and 1 MiB read
chunks, files without any newline, and the empty file.
"""
import os

import numpy as np
import pytest

import cases
import cmsbwt

pytestmark = pytest.mark.gpu


def _host(path):
    docs, sn = cmsbwt.host_read_collection(path)
    text = b"".join(d + b"\x02" for d in docs)
    off = np.zeros(len(docs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(d) + 1 for d in docs]) if docs else []
    return text, off, sn, sum(len(d) for d in docs), len(docs)


def _gpu(engine, path, env=None):
    env = dict(env or {})
    os.environ.update(env)
    try:
        engine.load_collection_file(path)
    finally:
        for k in env:
            os.environ.pop(k, None)
    text = engine.array("coll_text").tobytes()
    off = engine.array("coll_off")
    meta = engine.array("coll_meta")
    return text, off, int(meta[0]), int(meta[1]), int(meta[2])


def _check(engine, path, env=None):
    want = _host(path)
    got = _gpu(engine, path, env)
    assert got[4] == want[4], f"ndocs {got[4]} vs {want[4]}"
    assert np.array_equal(got[1], want[1]), "document offsets differ"
    if got[0] != want[0]:
        a = np.frombuffer(got[0], np.uint8)
        b = np.frombuffer(want[0], np.uint8)
        k = int(np.nonzero(a[: min(len(a), len(b))] != b[: min(len(a), len(b))])[0][:1].tolist() or [-1])
        raise AssertionError(f"text differs ({len(a)} vs {len(b)} bytes, first diff at {k})")
    assert got[2] == want[2], f"sn {got[2]} vs {want[2]}"
    assert got[3] == want[3]


def _ref_file(tmp_path, ref=b"ACGT" * 64):
    rp = str(tmp_path / "ref.fa")
    with open(rp, "wb") as f:
        f.write(b">r\n" + ref + b"\n")
    return rp


@pytest.mark.parametrize("case", [c for c in cases.small_cases() if c[3] == cases.UINT64_MAX], ids=lambda c: c[0])
def test_gpu_reader_small_cases(engine, tmp_path, case):
    d, rp, cp, _ = cases.materialise(tmp_path, case)
    engine.initialize_reference(rp)
    _check(engine, cp)


def _random_structured(rng, n_lines):
    """Lines of random widths (0 .. 40000, so lines straddle tiles), headers of
    random lengths (some longer than a tile), blank runs, CR bytes."""
    parts = []
    for _ in range(n_lines):
        r = rng.random()
        if r < 0.08:
            parts.append(b">" + b"h" * int(rng.integers(0, 20000)) + b"\n")
        elif r < 0.14:
            parts.append(b"\n" * int(rng.integers(1, 4)))
        else:
            w = int(rng.integers(0, 40000))
            s = cases.ACGT[rng.integers(0, 4, w)].tobytes()
            if rng.random() < 0.05:
                s += b"\r"
            parts.append(s + b"\n")
    return b"".join(parts)


@pytest.mark.parametrize("seed,tail", [(1, b""), (2, b"ACGTACG"), (3, b">unterminated header"), (4, b"\n")])
def test_gpu_reader_random_structure_multichunk(engine, tmp_path, seed, tail):
    rng = np.random.default_rng(seed)
    body = _random_structured(rng, 700) + tail
    if seed == 2:
        body = b"ACGT\n" + body  # headerless first document
    cp = str(tmp_path / "c.fa")
    with open(cp, "wb") as f:
        f.write(body)
    engine.initialize_reference(_ref_file(tmp_path))
    # 1 MiB chunks over 3 threads: chunk and thread boundaries fall inside lines
    _check(engine, cp, {"CMSBWT_READ_THREADS": "3", "CMSBWT_READ_CHUNK_MB": "1"})
    _check(engine, cp)


@pytest.mark.parametrize("body", [b"", b"ACGT", b">", b"\n", b"\n\n\n", b">a\n", b"A\n", b">x\nACGT\n>y\n",
                                  b"A" * 16383 + b"\n" + b">" + b"B" * 16384 + b"\nCC\n"],
                         ids=["empty", "no_newline", "gt_only", "nl", "nl3", "hdr", "one", "two_hdr", "tile_edge"])
def test_gpu_reader_degenerate(engine, tmp_path, body):
    cp = str(tmp_path / "c.fa")
    with open(cp, "wb") as f:
        f.write(body.replace(b"B", b"A"))
    engine.initialize_reference(_ref_file(tmp_path))
    _check(engine, cp)


def test_gpu_reader_rejects_foreign_byte_like_host(engine, tmp_path):
    cp = str(tmp_path / "c.fa")
    with open(cp, "wb") as f:
        f.write(b">a\nACGT\n>b\nAC\x80GT\nAC\x01GT\n")  # the augmentation adds 3..127 only (FN:231-237)
    engine.initialize_reference(_ref_file(tmp_path))
    with pytest.raises(cmsbwt.CmsBwtError) as e1:
        engine.load_collection_file(cp)
    os.environ["CMSBWT_HOST_READER"] = "1"
    try:
        with pytest.raises(cmsbwt.CmsBwtError) as e2:
            engine.load_collection_file(cp)
    finally:
        os.environ.pop("CMSBWT_HOST_READER")
    assert e1.value.code == e2.value.code == 3
    assert str(e1.value) == str(e2.value)


# ---- byte-range sharded ingest (cmsbwt_load_collection_file_range): each
# rank reads its slice of the file; the ranks' documents in rank order must be
# the whole file's (the getline semantics of FN:1138-1147 per slice)
def _range_docs(engine, path, rank, world):
    engine.load_collection_file_range(path, rank, world)
    text = engine.array("coll_text").tobytes()
    off = engine.array("coll_off")
    return [text[int(off[k]):int(off[k + 1]) - 1] for k in range(len(off) - 1)]


def _check_shards(engine, path, world):
    want, _ = cmsbwt.host_read_collection(path)
    got = []
    for k in range(world):
        got += _range_docs(engine, path, k, world)
    assert len(got) == len(want), f"{len(got)} vs {len(want)} documents at world {world}"
    assert got == want


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("case", [c for c in cases.small_cases() if c[3] == cases.UINT64_MAX], ids=lambda c: c[0])
def test_sharded_loader_small_cases(engine, tmp_path, case, world):
    d, rp, cp, _ = cases.materialise(tmp_path, case)
    engine.initialize_reference(rp)
    _check_shards(engine, cp, world)


@pytest.mark.parametrize("seed,tail", [(1, b""), (2, b"ACGTACG"), (3, b">unterminated header"), (4, b"\n")])
def test_sharded_loader_random_structure(engine, tmp_path, seed, tail):
    rng = np.random.default_rng(seed)
    body = _random_structured(rng, 700) + tail
    if seed == 2:
        body = b"ACGT\n" + body
    cp = str(tmp_path / "c.fa")
    with open(cp, "wb") as f:
        f.write(body)
    engine.initialize_reference(_ref_file(tmp_path))
    for world in (3, 7):
        _check_shards(engine, cp, world)


@pytest.mark.parametrize("body", [b"", b"ACGT", b">", b"\n", b"\n\n\n", b">a\n", b"A\n", b">x\nACGT\n>y\n",
                                  b"A" * 16383 + b"\n" + b">" + b"B" * 16384 + b"\nCC\n"],
                         ids=["empty", "no_newline", "gt_only", "nl", "nl3", "hdr", "one", "two_hdr", "tile_edge"])
def test_sharded_loader_degenerate(engine, tmp_path, body):
    """More ranks than documents: ranks own no document (empty slices)."""
    cp = str(tmp_path / "c.fa")
    with open(cp, "wb") as f:
        f.write(body.replace(b"B", b"A"))
    engine.initialize_reference(_ref_file(tmp_path))
    for world in (3, 5):
        _check_shards(engine, cp, world)
