"""GPU: the merge's scan and compaction primitives (merge.hip tile scan and
tile select, rocPRIM fallbacks behind CMSBWT_ROCPRIM_SCAN / _SELECT) against
host results, over tile edges (tiles of 2048 values), unaligned pointers and
in-place scans."""
import os

import pytest

pytestmark = pytest.mark.gpu

SIZES = [1, 2, 7, 2047, 2048, 2049, 3 * 2048 + 5, 1_000_003]


@pytest.mark.parametrize("rocprim", [False, True], ids=["tile", "rocprim"])
@pytest.mark.parametrize("what", ["exscan", "inscan", "select"])
def test_primitives_match_host(engine, what, rocprim):
    env = "CMSBWT_ROCPRIM_SELECT" if what == "select" else "CMSBWT_ROCPRIM_SCAN"
    os.environ[env] = "1" if rocprim else "0"
    try:
        for n in SIZES:
            for offset in (0, 1, 3):
                modes = (False,) if what == "select" else (False, True)
                for inplace in modes:
                    assert engine.selftest(what, n, offset, inplace) == 0, (what, n, offset, inplace)
    finally:
        os.environ.pop(env, None)


def test_select_refuses_in_place(engine):
    import cmsbwt
    with pytest.raises(cmsbwt.CmsBwtError) as e:
        engine.selftest("select", 100, 0, True)
    assert e.value.code == cmsbwt.CMSBWT_EARG
