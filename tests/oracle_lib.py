"""ctypes binding of the CPU oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg — never by the product package."""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
GEN = os.path.join(ROOT, "oracle", "_build", "gen_synth")
STAT_KEYS = ["heads", "positions", "keys", "rank", "current_sum", "bad", "good", "nothing", "runs", "D"]
DUMPS = {
    "h_start": "u4", "h_pos": "u4", "h_len": "u4", "h_smaller": "u1", "h_lchar": "u1", "h_isa": "u4",
    "h_tonext": "u4", "h_nexthead": "u2", "bucket": "i8", "rank2head": "i4", "head2rank": "i4",
    "bwtheads": "u1", "counters": "u8",
}
_ext = {"u4": "u32", "u1": "u8", "u2": "u16", "i8": "i64", "i4": "i32", "u8": "u64"}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError("oracle not built (make -C oracle)")
        _lib = ctypes.CDLL(LIB)
        _lib.oracle_run.restype = ctypes.c_int
        _lib.oracle_run.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                                    ctypes.c_ulonglong, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                    ctypes.POINTER(ctypes.c_ulonglong)]
    return _lib


def run(ref, coll, outname, rle=True, prefix=(1 << 64) - 1, dump_dir=None):
    """Run the oracle on files; returns (rc, stats dict, (t_index, t_collection))."""
    t = (ctypes.c_double * 2)()
    s = (ctypes.c_ulonglong * 10)()
    if dump_dir:
        os.makedirs(dump_dir, exist_ok=True)
    rc = lib().oracle_run(ref.encode(), coll.encode(), outname.encode(), 1 if rle else 0, prefix,
                          dump_dir.encode() if dump_dir else None, t, s)
    return rc, dict(zip(STAT_KEYS, list(s))), (t[0], t[1])


def load_dump(dump_dir, name):
    dt = DUMPS[name]
    return np.fromfile(os.path.join(dump_dir, f"{name}.{_ext[dt]}"), dtype=dt)
