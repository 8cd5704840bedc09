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
