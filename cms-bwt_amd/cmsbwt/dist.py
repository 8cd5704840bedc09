"""Document-sharded multi-GPU execution.

The MS walk and the j-scan are document-local (positions are per document,
FN:1149; the j-scan stops at the end-of-document phrase, FN:1367-1370), so
documents are sharded by contiguous ranges, one process per GPU.  The merge
is global: rank 0 gathers every shard's head records in document order
(= global idx order, because shards are contiguous and ordered), reduces the
per-position difference arrays (sum) and head flags (max), imports them and
runs the merge.  Transport is torch.distributed: RCCL ("nccl") over xGMI on
MI355X, gloo for the CPU tests.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from . import ARRAYS, WALK_ARRAYS

# wire dtypes (same bytes; RCCL has no unsigned 16/32-bit types)
_WIRE = {"u4": torch.int32, "i4": torch.int32, "u2": torch.int16, "u1": torch.uint8}
HEAD_ARRAYS = [a for a in WALK_ARRAYS if a.startswith("h_")]


def shard_range(total: int, world: int, rank: int):
    """Contiguous, balanced [begin, end) of `total` units for `rank`."""
    base, extra = divmod(total, world)
    b = rank * base + min(rank, extra)
    return b, b + base + (1 if rank < extra else 0)


def export_walk(eng, device) -> dict:
    """Copy this rank's walk results into torch tensors on `device`."""
    out = {}
    for name in WALK_ARRAYS:
        n = eng.array_size(name)
        t = torch.empty(n, dtype=_WIRE[ARRAYS[name]], device=device)
        if n:
            eng.array_into(name, t.data_ptr())
        out[name] = t
    if device != "cpu" and torch.cuda.is_available():
        torch.cuda.synchronize(device)
    return out


def gather_walk(local: dict, meta, device, root: int = 0):
    """Gather shards to `root`.  `local`: WALK_ARRAYS name -> 1-D tensor;
    meta: (heads, ndocs, chars) of this rank.  Returns (combined dict, totals)
    on root, (None, totals) elsewhere."""
    world, rank = dist.get_world_size(), dist.get_rank()
    meta = tuple(meta) + (1,) * (4 - len(meta))  # (heads, ndocs, chars, order_invariant)
    m = torch.tensor(list(meta), dtype=torch.int64, device=device)
    allm = [torch.zeros_like(m) for _ in range(world)]
    dist.all_gather(allm, m)
    sizes = [int(x[0]) for x in allm]
    totals = (sum(sizes), sum(int(x[1]) for x in allm), sum(int(x[2]) for x in allm),
              int(all(int(x[3]) for x in allm)))
    # per-position arrays: reduce to root
    diff = local["diff"].clone()
    hh = local["hashead"].clone()
    dist.reduce(diff, dst=root, op=dist.ReduceOp.SUM)
    dist.reduce(hh, dst=root, op=dist.ReduceOp.MAX)
    combined = None
    if rank == root:
        combined = {"diff": diff, "hashead": hh}
        offs = np.concatenate([[0], np.cumsum(sizes)])
        for name in HEAD_ARRAYS:
            buf = torch.empty(totals[0], dtype=local[name].dtype, device=device)
            buf[offs[rank]:offs[rank + 1]] = local[name]
            combined[name] = buf
    ops = []
    for name in HEAD_ARRAYS:
        if rank == root:
            for r in range(world):
                if r != root and sizes[r]:
                    ops.append(dist.P2POp(dist.irecv, combined[name][offs[r]:offs[r + 1]], r))
        elif sizes[rank]:
            ops.append(dist.P2POp(dist.isend, local[name], root))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return combined, totals


def import_walk(eng, combined: dict, totals):
    """Install gathered walk results into the merge rank's engine."""
    ptrs = [combined[name].data_ptr() for name in WALK_ARRAYS]
    eng.walk_import(totals[0], totals[1], totals[2], ptrs, order_invariant=bool(totals[3]))


def sharded_step(eng, device, rle: bool = True, root: int = 0):
    """One distributed step: local walk, gather, merge on root."""
    eng.ms_walk()
    st = eng.stats()
    local = export_walk(eng, device)
    combined, totals = gather_walk(local, (st.heads, st.ndocs, st.chars, st.order_invariant), device, root)
    if dist.get_rank() == root:
        import_walk(eng, combined, totals)
        eng.merge(rle)
    return totals
