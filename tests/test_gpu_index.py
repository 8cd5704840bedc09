"""Reference index on the GPU (ref_index.hip)
against the host build (SA-IS + Φ, host_index.cpp, itself checked against a
brute-force suffix sort in test_host.py): SA, ISA, LCP (with LCP[n] = -1),
the max-neighbour PLCP of FN:272-274 and the BWT must be identical, and so
must the walk tables built from them on the device (LCP block minima, child
table, adjacency records, prefix-rank tables) vs their host builds.
The references include long exact repeats and periodic strings (many
doubling rounds) and raw references with non-ACGT bytes."""
import os

import numpy as np
import pytest

import cases

pytestmark = pytest.mark.gpu

NAMES = ["ref_sa", "ref_isa", "ref_lcp", "ref_plcp", "ref_bwt",
         "ref_lvl", "ref_ld", "ref_pr", "ref_ir", "ref_pfx"]  # + the walk's tables (same layouts)


def _arrays(engine, ref, host):
    if host:
        os.environ["CMSBWT_HOST_INDEX"] = "1"
    try:
        engine.load_reference_bytes(ref)
    finally:
        os.environ.pop("CMSBWT_HOST_INDEX", None)
    return {k: engine.array(k) for k in NAMES}


def _refs():
    rng = np.random.default_rng(7)
    dna = cases.rand_dna(rng, 200_000)
    rep = dna[:50_000] * 3 + cases.mutate(rng, dna[:50_000], 0.01)
    return [
        ("tiny", b"A"),
        ("acgt", b"ACGT"),
        ("periodic", b"AC" * 40_000),
        ("homopolymer", b"A" * 70_000),
        ("random_200k", dna),
        ("repeats", rep),
        ("raw_with_N", cases.rand_dna(rng, 30_000).replace(b"AC", b"NN") + b"acgtRY" * 500),
        ("random_1m", cases.rand_dna(rng, 1_000_000)),
    ]


@pytest.mark.parametrize("name,ref", _refs(), ids=lambda v: v if isinstance(v, str) else "")
def test_gpu_index_equals_host_index(engine, name, ref):
    want = _arrays(engine, ref, host=True)
    got = _arrays(engine, ref, host=False)
    for k in NAMES:
        a, b = got[k], want[k]
        assert a.shape == b.shape, f"{name}: {k} shape"
        if not np.array_equal(a, b):
            bad = np.nonzero(a != b)[0]
            raise AssertionError(f"{name}: {k} differs at {len(bad)} entries, first {bad[:5]}")
