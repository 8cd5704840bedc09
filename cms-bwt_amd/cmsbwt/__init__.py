"""cmsbwt — Python mirror of the CMS-BWT operator surface over libcmsbwt.so.

The reference (fmasillo/CMS-BWT) exposes one entry point,
``computeBWT(Args, ref, coll)`` (CMS-BWT.h:69, CMS-BWT-functions.cpp:1788),
plus the ``cmsbwt`` CLI (main.cpp).  This module binds the C ABI declared in
``include/cmsbwt.h`` with ctypes and keeps the reference's names:

* :class:`Args`                  — utils.h:8-14 (filename/outname/format/buffer/prefixLength)
* :func:`computeBWT`             — CMS-BWT-functions.cpp:1788, raises instead of ``exit()``
* :class:`Engine`                — stage-level access (initialize_reference, ms_walk,
                                    merge, write) on one HIP device

The HIP library is mandatory: importing works without a GPU, but every
compute call goes through ``libcmsbwt.so`` and fails loudly if the library or
a device is missing.  There is no CPU fallback in this package.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field
from typing import Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
# CMSBWT_LIB selects another build of the same library (A/B experiments)
_LIB_PATH = os.environ.get("CMSBWT_LIB") or os.path.join(os.path.dirname(_HERE), "build", "libcmsbwt.so")

CMSBWT_OK = 0
CMSBWT_EIO = 1
CMSBWT_EARG = 2
CMSBWT_EINPUT = 3
CMSBWT_EDEVICE = 4
CMSBWT_ELIMIT = 5
CMSBWT_EORDER = 6
CMSBWT_EINTERNAL = 7
CMSBWT_BACKEND_PEER = 0
CMSBWT_BACKEND_RCCL = 1
UINT64_MAX = (1 << 64) - 1

ARRAYS = {  # name -> numpy dtype, as dumped by the oracle
    "ref_sa": "i4", "ref_isa": "u4", "ref_lcp": "i4", "ref_plcp": "i4", "ref_bwt": "u1",  # staged index
    "ref_ld": "u4", "ref_pr": "u4", "ref_ir": "u4", "ref_pfx": "u4", "ref_lvl": "i4",  # walk tables
    "coll_text": "u1", "coll_off": "u8", "coll_meta": "u8",  # loaded collection (text+seps, offsets, sn/chars/ndocs)
    "h_start": "u4", "h_pos": "u4", "h_len": "u4", "h_smaller": "u1", "h_lchar": "u1",
    "h_isa": "u4", "h_tonext": "u4", "h_nexthead": "u2", "bucket": "i8",
    "rank2head": "i4", "head2rank": "i4", "bwtheads": "u1", "counters": "u8",
    "diff": "i4", "hashead": "u1",
}
WALK_ARRAYS = ["h_start", "h_pos", "h_len", "h_smaller", "h_lchar", "h_isa", "h_tonext", "h_nexthead",
               "diff", "hashead"]


class CmsBwtError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"cmsbwt error {code}: {msg}")
        self.code = code


class _Args(ctypes.Structure):
    _fields_ = [("prefix", ctypes.c_uint64), ("buffer_gb", ctypes.c_uint32), ("rle", ctypes.c_int32),
                ("outname", ctypes.c_char_p), ("device", ctypes.c_int32), ("verbose", ctypes.c_int32),
                ("n_gpus", ctypes.c_int32), ("backend", ctypes.c_int32)]


class Stats(ctypes.Structure):
    _fields_ = [(k, ctypes.c_uint64) for k in (
        "n", "sn", "ndocs", "chars", "heads", "positions", "keys", "rank", "current_sum",
        "counter_bad", "counter_good", "counter_nothing", "runs", "symbols", "order_violations")] + \
        [(k, ctypes.c_double) for k in (
            "t_index_s", "t_upload_s", "t_ms_walk_s", "t_merge_s", "t_write_s", "ms_walk_kernel_ms",
            "counter_kernel_ms")] + [("counter_work", ctypes.c_uint64), ("order_invariant", ctypes.c_uint64)] + \
        [(k, ctypes.c_uint64) for k in ("ref_file_bytes", "ref_read_size", "coll_file_bytes", "sn_initial")] + \
        [(k, ctypes.c_int64) for k in ("first_rank_to_head", "last_rank_to_head")] + \
        [(k, ctypes.c_double) for k in ("t_augment_ms", "t_sa_ms", "t_isa_ms", "t_lcp_ms", "t_rmq_ms", "t_bwt_ms",
                                        "t_ranks_ms", "t_libsais_int_ms", "t_counter_ms")] + \
        [("host_queries", ctypes.c_uint64), ("device_peak_bytes", ctypes.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None


class RankTimes(ctypes.Structure):
    """include/cmsbwt.h cmsbwt_rank_times."""
    _fields_ = [(k, ctypes.c_double) for k in ("walk_ms", "merge_ms", "walk_kernel_ms")] + \
        [(k, ctypes.c_uint64) for k in ("heads", "chars", "device_peak_bytes")] + \
        [("gathered", ctypes.c_int32), ("device", ctypes.c_int32)]


def library_path() -> str:
    return _LIB_PATH


def load_library() -> ctypes.CDLL:
    """Load libcmsbwt.so (built by ``make lib``); raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        raise CmsBwtError(CMSBWT_EDEVICE, f"{_LIB_PATH} not built (run `make lib` or __graft_entry__.build())")
    # One HIP runtime per process: PyTorch ships its own libamdhip64.so.7 /
    # libhsa-runtime64.so.1 with the same sonames as /opt/rocm's.  Whichever
    # loads first serves both, and torch cannot initialise the GPU on a
    # runtime other than its own, so torch (when installed) goes first.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(_LIB_PATH)
    P, U64, I32, VP = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p
    sig = {
        "cmsbwt_run": (I32, [ctypes.POINTER(_Args), ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(Stats)]),
        "cmsbwt_run_sized": (I32, [ctypes.POINTER(_Args), U64, ctypes.c_char_p, ctypes.c_char_p,
                                   ctypes.POINTER(Stats), U64]),
        "cmsbwt_abi_version": (I32, []),
        "cmsbwt_ctx_create": (I32, [I32, ctypes.POINTER(P)]),
        "cmsbwt_ctx_destroy": (None, [P]),
        "cmsbwt_last_error": (ctypes.c_char_p, [P]),
        "cmsbwt_load_reference_file": (I32, [P, ctypes.c_char_p]),
        "cmsbwt_load_reference": (I32, [P, VP, U64]),
        "cmsbwt_load_collection_file": (I32, [P, ctypes.c_char_p, U64]),
        "cmsbwt_load_collection": (I32, [P, VP, VP, U64]),
        "cmsbwt_load_collection_file_range": (I32, [P, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32]),
        "cmsbwt_host_shard_bounds": (I32, [ctypes.c_char_p, ctypes.c_uint32, VP]),
        "cmsbwt_load_collection_synth": (I32, [P, U64, U64, U64, ctypes.c_double, I32]),
        "cmsbwt_ms_walk": (I32, [P]),
        "cmsbwt_merge": (I32, [P, I32]),
        "cmsbwt_step": (I32, [P, I32]),
        "cmsbwt_get_stats": (I32, [P, ctypes.POINTER(Stats)]),
        "cmsbwt_num_runs": (U64, [P]),
        "cmsbwt_copy_runs": (I32, [P, VP, U64]),
        "cmsbwt_write_output": (I32, [P, ctypes.c_char_p, I32]),
        "cmsbwt_copy_array": (I32, [P, ctypes.c_char_p, VP, ctypes.POINTER(U64)]),
        "cmsbwt_host_read_collection": (I32, [ctypes.c_char_p, U64, VP, U64, ctypes.POINTER(U64), VP, U64,
                                              ctypes.POINTER(U64), ctypes.POINTER(U64)]),
        "cmsbwt_host_suffix_array": (I32, [VP, U64, VP]),
        "cmsbwt_walk_import": (I32, [P, U64, U64, U64, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p)]),
        "cmsbwt_selftest": (I32, [P, ctypes.c_char_p, U64, U64, I32, ctypes.POINTER(U64)]),
        # position-sharded merge (device pointers; cmsbwt.dist drives the transport)
        "cmsbwt_dm_begin": (I32, [P, ctypes.c_uint32, ctypes.c_uint32, U64, U64, ctypes.c_uint32, I32]),
        "cmsbwt_dm_route_heads": (I32, [P, VP]),
        "cmsbwt_dm_pack_heads": (I32, [P, VP]),
        "cmsbwt_dm_group": (I32, [P, VP, U64, VP]),
        "cmsbwt_dm_labels": (I32, [P, VP, VP]),
        "cmsbwt_dm_dbl_init": (I32, [P, VP, ctypes.POINTER(U64)]),
        "cmsbwt_dm_dbl_route": (I32, [P, U64, VP]),
        "cmsbwt_dm_dbl_pack": (I32, [P, VP]),
        "cmsbwt_dm_dbl_sort": (I32, [P, VP, U64, VP]),
        "cmsbwt_dm_dbl_apply": (I32, [P, VP, ctypes.POINTER(U64)]),
        "cmsbwt_dm_pack_ranks": (I32, [P, VP]),
        "cmsbwt_dm_load_ranks": (I32, [P, VP]),
        "cmsbwt_dm_route_halo": (I32, [P, VP, VP]),
        "cmsbwt_dm_pack_halo": (I32, [P, VP, VP]),
        "cmsbwt_dm_counter": (I32, [P, VP, U64, VP, U64, VP]),
        "cmsbwt_dm_units": (I32, [P, VP]),
        "cmsbwt_dm_emit": (I32, [P, VP, ctypes.POINTER(U64)]),
        "cmsbwt_dm_copy_stream": (I32, [P, VP, VP]),
        "cmsbwt_dm_finish": (I32, [P, ctypes.POINTER(VP), ctypes.POINTER(VP), VP, VP]),
        # rank groups (in-process multi-GPU step over resident inputs)
        "cmsbwt_group_create": (I32, [I32, I32, I32, ctypes.POINTER(P)]),
        "cmsbwt_group_ctx": (P, [P, I32]),
        "cmsbwt_group_step": (I32, [P, I32, ctypes.POINTER(RankTimes)]),
        "cmsbwt_group_last_error": (ctypes.c_char_p, [P]),
        "cmsbwt_group_destroy": (None, [P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


EXPORTED = [
    "cmsbwt_run", "cmsbwt_run_sized", "cmsbwt_abi_version", "cmsbwt_ctx_create", "cmsbwt_ctx_destroy", "cmsbwt_last_error",
    "cmsbwt_load_reference_file", "cmsbwt_load_reference", "cmsbwt_load_collection_file",
    "cmsbwt_load_collection", "cmsbwt_load_collection_synth", "cmsbwt_ms_walk", "cmsbwt_merge",
    "cmsbwt_step", "cmsbwt_get_stats", "cmsbwt_num_runs", "cmsbwt_copy_runs", "cmsbwt_write_output",
    "cmsbwt_copy_array", "cmsbwt_host_read_collection", "cmsbwt_host_suffix_array", "cmsbwt_walk_import",
    "cmsbwt_selftest", "cmsbwt_load_collection_file_range", "cmsbwt_host_shard_bounds",
    "cmsbwt_dm_begin", "cmsbwt_dm_route_heads", "cmsbwt_dm_pack_heads", "cmsbwt_dm_group", "cmsbwt_dm_labels",
    "cmsbwt_dm_dbl_init", "cmsbwt_dm_dbl_route", "cmsbwt_dm_dbl_pack", "cmsbwt_dm_dbl_sort", "cmsbwt_dm_dbl_apply",
    "cmsbwt_dm_pack_ranks", "cmsbwt_dm_load_ranks", "cmsbwt_dm_route_halo", "cmsbwt_dm_pack_halo",
    "cmsbwt_dm_counter", "cmsbwt_dm_units", "cmsbwt_dm_emit", "cmsbwt_dm_copy_stream", "cmsbwt_dm_finish",
    "cmsbwt_group_create", "cmsbwt_group_ctx", "cmsbwt_group_step", "cmsbwt_group_last_error",
    "cmsbwt_group_destroy",
]


@dataclass
class Args:
    """utils.h:8-14."""
    filename: str = ""
    outname: str = ""
    format: bool = False          # -r : run-length encoded output
    buffer: int = 2               # -b
    prefixLength: int = UINT64_MAX  # -p
    device: int = 0
    verbose: bool = False
    n_gpus: int = 1               # ranks in this process (include/cmsbwt.h cmsbwt_args)
    backend: str = "peer"         # multi-GPU transport: "peer" | "rccl"


def computeBWT(arg: Args, refFileName: str, collFileName: str) -> Stats:
    """CMS-BWT-functions.cpp:1788-1797 — writes <outname>.rl_bwt|.bwt and .log.

    Raises :class:`CmsBwtError` where the reference would ``exit()``."""
    lib = load_library()
    out = arg.outname or arg.filename
    a = _Args(arg.prefixLength, arg.buffer, 1 if arg.format else 0, out.encode(), arg.device,
              1 if arg.verbose else 0, arg.n_gpus,
              CMSBWT_BACKEND_RCCL if arg.backend == "rccl" else CMSBWT_BACKEND_PEER)
    st = Stats()
    rc = lib.cmsbwt_run_sized(ctypes.byref(a), ctypes.sizeof(a), refFileName.encode(), collFileName.encode(),
                              ctypes.byref(st), ctypes.sizeof(st))
    if rc != CMSBWT_OK:
        raise CmsBwtError(rc, f"computeBWT failed, see {out}.log")
    return st


class Engine:
    """One HIP device context; stages of the hot path callable one by one."""

    def __init__(self, device: int = 0):
        self._lib = load_library()
        p = ctypes.c_void_p()
        rc = self._lib.cmsbwt_ctx_create(device, ctypes.byref(p))
        if rc != CMSBWT_OK:
            raise CmsBwtError(rc, f"no usable HIP device {device}")
        self._ctx = p

    def close(self):
        if self._ctx and not getattr(self, "_borrowed", False):
            self._lib.cmsbwt_ctx_destroy(self._ctx)
        self._ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc: int):
        if rc != CMSBWT_OK:
            raise CmsBwtError(rc, self._lib.cmsbwt_last_error(self._ctx).decode(errors="replace"))

    # initialize_reference (FN:151-310)
    def initialize_reference(self, path: str):
        self._chk(self._lib.cmsbwt_load_reference_file(self._ctx, path.encode()))

    def load_reference_bytes(self, ref: bytes):
        buf = ctypes.create_string_buffer(ref, len(ref))
        self._chk(self._lib.cmsbwt_load_reference(self._ctx, buf, len(ref)))

    def load_collection_file(self, path: str, prefix: int = UINT64_MAX):
        self._chk(self._lib.cmsbwt_load_collection_file(self._ctx, path.encode(), prefix))

    def load_collection_file_range(self, path: str, rank: int, world: int):
        """This rank's documents of the collection file (byte-range shards,
        cmsbwt_host_shard_bounds), read on the device."""
        self._chk(self._lib.cmsbwt_load_collection_file_range(self._ctx, path.encode(), rank, world))

    def load_collection(self, docs):
        import numpy as np
        text = b"".join(docs)
        off = np.zeros(len(docs) + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(d) for d in docs])
        buf = ctypes.create_string_buffer(text, max(1, len(text)))
        self._chk(self._lib.cmsbwt_load_collection(self._ctx, buf, off.ctypes.data, len(docs)))

    def load_collection_array(self, text, doc_off):
        """Documents from a contiguous uint8 numpy array and uint64 offsets
        (doc k = text[doc_off[k]:doc_off[k+1]]), without intermediate copies."""
        import numpy as np
        text = np.ascontiguousarray(text, dtype=np.uint8)
        off = np.ascontiguousarray(doc_off, dtype=np.uint64)
        self._chk(self._lib.cmsbwt_load_collection(self._ctx, text.ctypes.data if text.size else None,
                                                   off.ctypes.data, len(off) - 1))

    def load_synth(self, seed: int, copy_begin: int, ncopies: int, p: float, leading_empty_doc: bool = True):
        self._chk(self._lib.cmsbwt_load_collection_synth(self._ctx, seed, copy_begin, ncopies, p,
                                                         1 if leading_empty_doc else 0))

    def ms_walk(self):
        self._chk(self._lib.cmsbwt_ms_walk(self._ctx))

    def merge(self, rle: bool = True):
        self._chk(self._lib.cmsbwt_merge(self._ctx, 1 if rle else 0))

    def step(self, rle: bool = True):
        self._chk(self._lib.cmsbwt_step(self._ctx, 1 if rle else 0))

    def stats(self) -> Stats:
        st = Stats()
        self._chk(self._lib.cmsbwt_get_stats(self._ctx, ctypes.byref(st)))
        return st

    def runs_bytes(self) -> bytes:
        nr = self._lib.cmsbwt_num_runs(self._ctx)
        buf = ctypes.create_string_buffer(max(1, nr * 9))
        self._chk(self._lib.cmsbwt_copy_runs(self._ctx, buf, nr * 9))
        return buf.raw[: nr * 9]

    def array_size(self, name: str) -> int:
        nb = ctypes.c_uint64()
        self._chk(self._lib.cmsbwt_copy_array(self._ctx, name.encode(), None, ctypes.byref(nb)))
        return nb.value // __import__("numpy").dtype(ARRAYS[name]).itemsize

    def array_into(self, name: str, ptr: int):
        """Copy a stage array into caller memory (host or device pointer)."""
        nb = ctypes.c_uint64()
        self._chk(self._lib.cmsbwt_copy_array(self._ctx, name.encode(), ctypes.c_void_p(ptr), ctypes.byref(nb)))

    def walk_import(self, heads: int, ndocs: int, chars: int, ptrs, order_invariant: bool = False):
        """Install merged walk results (pointers in WALK_ARRAYS order, host or device)."""
        arr = (ctypes.c_void_p * len(WALK_ARRAYS))(*[ctypes.c_void_p(p) for p in ptrs])
        self._chk(self._lib.cmsbwt_walk_import(self._ctx, heads, ndocs, chars, 1 if order_invariant else 0, arr))

    # ---- position-sharded merge: thin wrappers, pointers are device addresses
    # (ints, e.g. torch.Tensor.data_ptr()); see include/cmsbwt.h for the order
    def _u64s(self, k):
        return (ctypes.c_uint64 * k)()

    def dm_begin(self, world, rank, heads_total, docs_total, order_invariant, rle=True):
        self._chk(self._lib.cmsbwt_dm_begin(self._ctx, world, rank, heads_total, docs_total,
                                            1 if order_invariant else 0, 1 if rle else 0))

    def dm_route_heads(self, world):
        c = self._u64s(world)
        self._chk(self._lib.cmsbwt_dm_route_heads(self._ctx, c))
        return list(c)

    def dm_pack_heads(self, out_ptr):
        self._chk(self._lib.cmsbwt_dm_pack_heads(self._ctx, ctypes.c_void_p(out_ptr)))

    def dm_group(self, recv_ptr, nrecv, sa_counts_ptr):
        self._chk(self._lib.cmsbwt_dm_group(self._ctx, ctypes.c_void_p(recv_ptr), nrecv,
                                            ctypes.c_void_p(sa_counts_ptr)))

    def dm_labels(self, sa_counts_ptr, back_ptr):
        self._chk(self._lib.cmsbwt_dm_labels(self._ctx, ctypes.c_void_p(sa_counts_ptr), ctypes.c_void_p(back_ptr)))

    def dm_dbl_init(self, labels_ptr):
        a = ctypes.c_uint64()
        self._chk(self._lib.cmsbwt_dm_dbl_init(self._ctx, ctypes.c_void_p(labels_ptr), ctypes.byref(a)))
        return a.value

    def dm_dbl_route(self, h, world):
        c = self._u64s(world)
        self._chk(self._lib.cmsbwt_dm_dbl_route(self._ctx, h, c))
        return list(c)

    def dm_dbl_pack(self, out_ptr):
        self._chk(self._lib.cmsbwt_dm_dbl_pack(self._ctx, ctypes.c_void_p(out_ptr)))

    def dm_dbl_sort(self, recv_ptr, nrecv, res_ptr):
        self._chk(self._lib.cmsbwt_dm_dbl_sort(self._ctx, ctypes.c_void_p(recv_ptr), nrecv, ctypes.c_void_p(res_ptr)))

    def dm_dbl_apply(self, back_ptr):
        a = ctypes.c_uint64()
        self._chk(self._lib.cmsbwt_dm_dbl_apply(self._ctx, ctypes.c_void_p(back_ptr), ctypes.byref(a)))
        return a.value

    def dm_pack_ranks(self, out_ptr):
        self._chk(self._lib.cmsbwt_dm_pack_ranks(self._ctx, ctypes.c_void_p(out_ptr)))

    def dm_load_ranks(self, recv_ptr):
        self._chk(self._lib.cmsbwt_dm_load_ranks(self._ctx, ctypes.c_void_p(recv_ptr)))

    def dm_route_halo(self, world):
        ic, wc = self._u64s(world), self._u64s(world)
        self._chk(self._lib.cmsbwt_dm_route_halo(self._ctx, ic, wc))
        return list(ic), list(wc)

    def dm_pack_halo(self, hdr_ptr, words_ptr):
        self._chk(self._lib.cmsbwt_dm_pack_halo(self._ctx, ctypes.c_void_p(hdr_ptr), ctypes.c_void_p(words_ptr)))

    def dm_counter(self, hdr_ptr, nitems, words_ptr, nwords):
        """-> [bad, good, nothing, violations, errors, items] of this rank."""
        out = self._u64s(6)
        self._chk(self._lib.cmsbwt_dm_counter(self._ctx, ctypes.c_void_p(hdr_ptr), nitems, ctypes.c_void_p(words_ptr),
                                              nwords, out))
        return list(out)

    def dm_units(self, units_ptr):
        self._chk(self._lib.cmsbwt_dm_units(self._ctx, ctypes.c_void_p(units_ptr)))

    def dm_emit(self, units_ptr):
        a = ctypes.c_uint64()
        self._chk(self._lib.cmsbwt_dm_emit(self._ctx, ctypes.c_void_p(units_ptr), ctypes.byref(a)))
        return a.value

    def dm_copy_stream(self, starts_ptr, chars_ptr):
        self._chk(self._lib.cmsbwt_dm_copy_stream(self._ctx, ctypes.c_void_p(starts_ptr), ctypes.c_void_p(chars_ptr)))

    def dm_finish(self, start_ptrs, char_ptrs, counts, gstats):
        k = len(counts)
        sp = (ctypes.c_void_p * k)(*[ctypes.c_void_p(p) for p in start_ptrs])
        cp = (ctypes.c_void_p * k)(*[ctypes.c_void_p(p) for p in char_ptrs])
        cn = (ctypes.c_uint64 * k)(*counts)
        gs = (ctypes.c_uint64 * len(gstats))(*gstats)
        self._chk(self._lib.cmsbwt_dm_finish(self._ctx, sp, cp, cn, gs))

    def selftest(self, what: str, n: int, offset: int = 0, inplace: bool = False) -> int:
        """Mismatches of a device primitive against its host result (0 = equal)."""
        bad = ctypes.c_uint64()
        self._chk(self._lib.cmsbwt_selftest(self._ctx, what.encode(), n, offset, 1 if inplace else 0,
                                            ctypes.byref(bad)))
        return bad.value

    def write_output(self, outname: str, rle: bool = True):
        self._chk(self._lib.cmsbwt_write_output(self._ctx, outname.encode(), 1 if rle else 0))

    def array(self, name: str):
        import numpy as np
        nb = ctypes.c_uint64()
        self._chk(self._lib.cmsbwt_copy_array(self._ctx, name.encode(), None, ctypes.byref(nb)))
        out = np.empty(nb.value // np.dtype(ARRAYS[name]).itemsize, dtype=ARRAYS[name])
        self._chk(self._lib.cmsbwt_copy_array(self._ctx, name.encode(), out.ctypes.data if out.size else None,
                                              ctypes.byref(nb)))
        return out


class Group:
    """`world` rank contexts in this process (include/cmsbwt.h "Rank groups"):
    rank k on device (device + k) % devices.  Load each rank through
    ``engine(k)`` (the ranks' documents, in rank order, are the collection),
    then ``step()`` runs every rank's walk and the position-sharded merge;
    the runs and the global statistics end up in ``engine(0)``."""

    def __init__(self, world: int, device: int = 0, backend: str = "peer"):
        self._lib = load_library()
        p = ctypes.c_void_p()
        rc = self._lib.cmsbwt_group_create(world, device, CMSBWT_BACKEND_RCCL if backend == "rccl"
                                           else CMSBWT_BACKEND_PEER, ctypes.byref(p))
        if rc != CMSBWT_OK:
            raise CmsBwtError(rc, f"cannot create a group of {world} ranks on device {device} ({backend})")
        self._g = p
        self.world = world
        self._engines = []
        for k in range(world):
            e = Engine.__new__(Engine)  # a view of the group's context (the group owns it)
            e._lib = self._lib
            e._ctx = ctypes.c_void_p(self._lib.cmsbwt_group_ctx(p, k))
            e._borrowed = True
            self._engines.append(e)

    def engine(self, rank: int) -> "Engine":
        return self._engines[rank]

    def step(self, rle: bool = True):
        """One walk + sharded merge on every rank; returns the per-rank RankTimes."""
        t = (RankTimes * self.world)()
        rc = self._lib.cmsbwt_group_step(self._g, 1 if rle else 0, t)
        if rc != CMSBWT_OK:
            raise CmsBwtError(rc, self._lib.cmsbwt_group_last_error(self._g).decode(errors="replace"))
        return list(t)

    def close(self):
        if self._g:
            for e in self._engines:
                e._ctx = None
            self._lib.cmsbwt_group_destroy(self._g)
            self._g = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def host_read_collection(path: str, prefix: int = UINT64_MAX):
    """Reader only (no GPU): returns (list of document bytes, sn)."""
    import numpy as np
    lib = load_library()
    tl, nd, sn = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    rc = lib.cmsbwt_host_read_collection(path.encode(), prefix, None, 0, ctypes.byref(tl), None, 0,
                                         ctypes.byref(nd), ctypes.byref(sn))
    if rc:
        raise CmsBwtError(rc, f"cannot read {path}")
    text = ctypes.create_string_buffer(max(1, tl.value))
    off = np.zeros(nd.value + 1, dtype=np.uint64)
    rc = lib.cmsbwt_host_read_collection(path.encode(), prefix, text, tl.value, ctypes.byref(tl),
                                         off.ctypes.data, nd.value + 1, ctypes.byref(nd), ctypes.byref(sn))
    if rc:
        raise CmsBwtError(rc, f"cannot read {path}")
    raw = text.raw
    return [raw[int(off[k]):int(off[k + 1])] for k in range(nd.value)], sn.value


def host_shard_bounds(path: str, world: int):
    """Byte bounds of the collection shards (no GPU needed)."""
    import numpy as np
    lib = load_library()
    out = np.zeros(world + 1, dtype=np.uint64)
    rc = lib.cmsbwt_host_shard_bounds(path.encode(), world, out.ctypes.data)
    if rc:
        raise CmsBwtError(rc, f"cannot shard {path}")
    return [int(x) for x in out]


def host_suffix_array(s: bytes):
    import numpy as np
    lib = load_library()
    out = np.empty(len(s), dtype=np.int32)
    buf = ctypes.create_string_buffer(s, max(1, len(s)))
    rc = lib.cmsbwt_host_suffix_array(buf, len(s), out.ctypes.data if len(s) else None)
    if rc:
        raise CmsBwtError(rc, "suffix array failed")
    return out


def decode_rl(raw: bytes):
    """(lengths uint64, chars uint8) of a .rl_bwt byte string (FN:1708-1709 records)."""
    import numpy as np
    a = np.frombuffer(raw, dtype=np.uint8).reshape(-1, 9)
    return a[:, :8].copy().view("<u8").ravel(), a[:, 8].copy()
