"""Multi-GPU execution.

The MS walk and the j-scan are document-local (positions are per document,
FN:1149; the j-scan stops at the end-of-document phrase, FN:1367-1370), so
documents are sharded by contiguous ranges, one process per GPU.  The merge
is global; two ways to run it:

* :func:`sharded_step` (default) — the merge sharded by reference position
  (dist_merge.hip): heads go to the owner of their position (all-to-all), the
  head-string suffix sort runs as distributed prefix doubling, counters and
  writer units are computed per position range, and rank 0 only places the
  runs every rank emitted and packs the records.
* :func:`gather_step` — rank 0 gathers every shard's head records in document
  order (= global idx order, shards being contiguous and ordered), reduces the
  per-position difference arrays (sum) and head flags (max), imports them and
  runs the single-GPU merge.

Transport is torch.distributed: RCCL ("nccl") over xGMI on MI355X, gloo (host
staging) for the CPU tests and for several ranks sharing one test GPU.
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
    # RCCL collectives and the root's slice copy are ordered on torch's current
    # stream only; the engine reads the tensors from its own stream, so the
    # host waits for them here (as Transport.sync does in the sharded merge).
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)
    return combined, totals


def import_walk(eng, combined: dict, totals):
    """Install gathered walk results into the merge rank's engine."""
    ptrs = [combined[name].data_ptr() for name in WALK_ARRAYS]
    eng.walk_import(totals[0], totals[1], totals[2], ptrs, order_invariant=bool(totals[3]))


def gather_step(eng, device, rle: bool = True, root: int = 0):
    """One distributed step: local walk, gather, merge on root."""
    eng.ms_walk()
    return gather_merge(eng, device, rle, root)


def gather_merge(eng, device, rle: bool = True, root: int = 0):
    """The merge of gather_step after this rank's walk: gather, merge on root."""
    st = eng.stats()
    local = export_walk(eng, device)
    combined, totals = gather_walk(local, (st.heads, st.ndocs, st.chars, st.order_invariant), device, root)
    if dist.get_rank() == root:
        import_walk(eng, combined, totals)
        eng.merge(rle)
    return totals


# ---------------------------------------------------------------- sharded merge
class Transport:
    """Collectives on 1-D/2-D device tensors (dim-0 splits).  With gloo and
    device tensors the data is staged through host memory; world == 1 needs no
    process group (identity exchange)."""

    def __init__(self, device, world=None, rank=None):
        self.device = torch.device(device)
        if world is None:
            world, rank = (dist.get_world_size(), dist.get_rank()) if dist.is_initialized() else (1, 0)
        self.world, self.rank = world, rank
        self.staged = self.world > 1 and dist.get_backend() == "gloo" and self.device.type != "cpu"

    def sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def empty(self, shape, dtype):
        return torch.empty(shape, dtype=dtype, device=self.device)

    def counts(self, send_counts):
        """Per-destination counts -> per-source counts."""
        if self.world == 1:
            return list(send_counts)
        t = torch.tensor(send_counts, dtype=torch.int64)
        out = torch.empty_like(t)
        if not self.staged and self.device.type != "cpu":
            t, out = t.to(self.device), out.to(self.device)
        dist.all_to_all_single(out, t)
        return [int(x) for x in out.tolist()]

    def a2a(self, send, send_counts, recv_counts):
        if self.world == 1:
            return send
        shape = (sum(recv_counts),) + tuple(send.shape[1:])
        if self.staged:
            out = torch.empty(shape, dtype=send.dtype)
            dist.all_to_all_single(out, send.cpu(), list(recv_counts), list(send_counts))
            out = out.to(self.device)
        else:
            out = torch.empty(shape, dtype=send.dtype, device=send.device)
            dist.all_to_all_single(out, send, list(recv_counts), list(send_counts))
        self.sync()
        return out

    def allreduce(self, t, op="sum"):
        if self.world == 1:
            return t
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX}[op]
        if self.staged:
            c = t.cpu()
            dist.all_reduce(c, op=rop)
            t.copy_(c)
        else:
            dist.all_reduce(t, op=rop)
        self.sync()
        return t

    def counts_and_sum(self, send_counts, value):
        """counts() plus the sum of `value` over all ranks, in one exchange."""
        if self.world == 1:
            return list(send_counts), int(value)
        t = torch.tensor([[c, value] for c in send_counts], dtype=torch.int64)
        out = torch.empty_like(t)
        if not self.staged and self.device.type != "cpu":
            t, out = t.to(self.device), out.to(self.device)
        dist.all_to_all_single(out, t)
        v = out.tolist()
        return [int(a) for a, _ in v], sum(int(b) for _, b in v)

    def allgather_ints(self, vals):
        """[per-rank list of ints] for a list of ints of equal length."""
        if self.world == 1:
            return [list(vals)]
        t = torch.tensor(vals, dtype=torch.int64)
        if not self.staged and self.device.type != "cpu":
            t = t.to(self.device)
        outs = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(outs, t)
        return [[int(x) for x in o.tolist()] for o in outs]


def sharded_step(eng, device, rle: bool = True, xfer: Transport = None):
    """One distributed step with the position-sharded merge (see module doc and
    include/cmsbwt.h "Multi-GPU merge").  The runs end up on rank 0."""
    eng.ms_walk()
    return sharded_merge(eng, xfer or Transport(device), rle)


class _StageClock:
    """CMSBWT_DM_TIMING=1: host wall time between the marks (stderr)."""

    def __init__(self, rank):
        import os
        import time
        self.on = os.environ.get("CMSBWT_DM_TIMING") == "1"
        self.rank, self._time, self.t, self.parts = rank, time.perf_counter, time.perf_counter(), []

    def mark(self, what):
        if self.on:
            t = self._time()
            self.parts.append(f"{what} {1e3 * (t - self.t):.2f}")
            self.t = t

    def flush(self):
        if self.on:
            import sys
            print(f"[py-dm-timing] rank {self.rank}: " + " ".join(self.parts), file=sys.stderr, flush=True)


def sharded_merge(eng, x: Transport, rle: bool = True):
    from . import CMSBWT_EINPUT, CmsBwtError
    world, rank = x.world, x.rank
    clk = _StageClock(rank)
    st = eng.stats()
    H, n = int(st.heads), int(st.n)
    meta = x.allgather_ints([H, int(st.ndocs), int(st.chars), int(st.order_invariant)])
    Htot = sum(m[0] for m in meta)
    E = sum(m[1] for m in meta)
    chars = sum(m[2] for m in meta)
    inv = all(m[3] for m in meta)
    i32, i64 = torch.int32, torch.int64
    eng.dm_begin(world, rank, Htot, E, inv, rle)
    clk.mark("meta+begin")
    # 1-2. heads to position owners; items; initial group labels
    hc = eng.dm_route_heads(world)
    send = x.empty((H, 5), i32)
    eng.dm_pack_heads(send.data_ptr())
    rc = x.counts(hc)
    recv = x.a2a(send, hc, rc)
    clk.mark("route+pack+a2a")
    del send
    Hp = sum(rc)
    # per-SA-rank item / head counts and the run difference array, one all-reduce
    sa = x.empty(3 * n + 1, i32)
    eng.dm_group(recv.data_ptr(), Hp, sa.data_ptr())
    del recv
    x.allreduce(sa, "sum")
    clk.mark("group+allreduce")
    back = x.empty(Hp, i64)  # label | unresolved << 32 (labels use all 32 bits)
    eng.dm_labels(sa.data_ptr(), back.data_ptr())
    del sa
    labels = x.a2a(back, rc, hc)
    U = eng.dm_dbl_init(labels.data_ptr())
    clk.mark("labels+dbl_init")
    del back, labels
    # 3. prefix doubling of the head string (one count exchange per round
    # also sums the unresolved members over ranks)
    h = 1
    while True:
        c = eng.dm_dbl_route(h, world)
        r, active = x.counts_and_sum(c, U)
        if active == 0:
            break
        send = x.empty((U, 2), i32)
        eng.dm_dbl_pack(send.data_ptr())
        recv = x.a2a(send, c, r)
        res = x.empty(sum(r), i64)
        eng.dm_dbl_sort(recv.data_ptr(), sum(r), res.data_ptr())
        back = x.a2a(res, r, c)
        U = eng.dm_dbl_apply(back.data_ptr())
        h *= 2
    clk.mark("doubling")
    # 4. head ranks / next-head ranks to the position owners
    ranks = x.empty((H, 3), i32)  # head rank, next-head rank, BWT character
    eng.dm_pack_ranks(ranks.data_ptr())
    rr = x.a2a(ranks, hc, rc)
    eng.dm_load_ranks(rr.data_ptr())
    clk.mark("ranks")
    del ranks, rr
    # 5. counters with the halo of items reaching in from earlier ranks
    ic, wc = eng.dm_route_halo(world)
    hdr = x.empty((sum(ic), 6), i32)
    words = x.empty(sum(wc), i32)
    eng.dm_pack_halo(hdr.data_ptr(), words.data_ptr())
    ric, rwc = x.counts(ic), x.counts(wc)
    hin = x.a2a(hdr, ic, ric)
    win = x.a2a(words, wc, rwc)
    c6 = eng.dm_counter(hin.data_ptr(), sum(ric), win.data_ptr(), sum(rwc))
    clk.mark("halo+counter")
    del hdr, words, hin, win
    g = x.allgather_ints(c6)
    bad, good, nothing, viol, errs, keys = [sum(v[k] for v in g) for k in range(6)]
    if errs:
        raise CmsBwtError(CMSBWT_EINPUT, "counter target beyond the reference (reference UB)")
    if viol:
        # match.h:27-33 is not a strict weak order on this input (DESIGN.md
        # §5).  The std::map replay that reproduces the reference's layout
        # runs in the one-GPU merge, so the step is redone as a gather step:
        # walk again, every head to rank 0, merge there.
        eng.ms_walk()
        if world == 1:
            eng.merge(rle)
            return Htot, E, chars
        dev = "cpu" if x.staged else x.device
        st = eng.stats()
        local = export_walk(eng, dev)
        combined, totals = gather_walk(local, (st.heads, st.ndocs, st.chars, st.order_invariant), dev, 0)
        if rank == 0:
            import_walk(eng, combined, totals)
            eng.merge(rle)
        return Htot, E, chars
    # 6. writer units, emission, gather to rank 0
    Uw = E + n - 1
    units = x.empty(2 * Uw, i64)
    eng.dm_units(units.data_ptr())
    x.allreduce(units, "sum")
    nloc = eng.dm_emit(units.data_ptr())
    clk.mark("units+emit")
    del units
    starts = x.empty(nloc, i64)
    chs = x.empty(nloc, torch.uint8)
    eng.dm_copy_stream(starts.data_ptr(), chs.data_ptr())
    counts = [v[0] for v in x.allgather_ints([nloc])]
    sc = [nloc if k == 0 else 0 for k in range(world)]
    rcv = counts if rank == 0 else [0] * world
    gst = x.a2a(starts, sc, rcv)
    gch = x.a2a(chs, sc, rcv)
    if rank == 0:
        offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        sp = [gst.data_ptr() + 8 * int(offs[k]) for k in range(world)]
        cp = [gch.data_ptr() + int(offs[k]) for k in range(world)]
        eng.dm_finish(sp, cp, counts, [Htot, keys, E, chars, bad, good, nothing, viol])
    clk.mark("gather+finish")
    clk.flush()
    return Htot, E, chars
