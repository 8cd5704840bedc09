"""Worker processes for the multi-rank tests (spawned by tests/test_multirank.py
and tests/test_gpu_dist.py).  Rendezvous on 127.0.0.1, gloo backend."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cms-bwt_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _init(rank, world, port, backend="gloo"):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if backend == "nccl":
        import torch
        torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)
    return dist


def cpu_gather(rank, world, port, work):
    """Each rank loads its shard's oracle dumps as walk results; rank 0 checks
    the gathered arrays against the global oracle dumps."""
    import torch
    import cmsbwt.dist as cdist
    import oracle_lib
    from cmsbwt import ARRAYS
    dist = _init(rank, world, port)
    cfg = json.load(open(os.path.join(work, "cfg.json")))
    sd = os.path.join(work, f"shard{rank}")
    local = {}
    for name in cdist.HEAD_ARRAYS:
        a = oracle_lib.load_dump(sd, name)
        local[name] = torch.from_numpy(a.view(np.dtype(ARRAYS[name]).newbyteorder("=")).copy()).view(
            cdist._WIRE[ARRAYS[name]])
    b = oracle_lib.load_dump(sd, "bucket")
    count = np.abs(b).astype(np.int64)
    diff = np.diff(np.concatenate([[0], count, [0]])).astype(np.int32)
    local["diff"] = torch.from_numpy(diff)
    local["hashead"] = torch.from_numpy((b < 0).astype(np.uint8))
    meta = (len(local["h_pos"]), cfg["ndocs"][rank], cfg["chars"][rank])
    combined, totals = cdist.gather_walk(local, meta, "cpu")
    if rank == 0:
        gd = os.path.join(work, "global")
        for name in cdist.HEAD_ARRAYS:
            want = oracle_lib.load_dump(gd, name)
            got = combined[name].numpy().view(ARRAYS[name])
            assert np.array_equal(got, want), name
        gb = oracle_lib.load_dump(gd, "bucket")
        cnt = np.cumsum(combined["diff"].numpy().astype(np.int64))[:-1]
        assert np.array_equal(np.where(combined["hashead"].numpy() > 0, -cnt, cnt), gb)
        nh = sum(len(oracle_lib.load_dump(os.path.join(work, f"shard{r}"), "h_pos")) for r in range(world))
        assert totals[:3] == (nh, sum(cfg["ndocs"]), sum(cfg["chars"]))
        open(os.path.join(work, "ok"), "w").write("ok")
    dist.destroy_process_group()


def gpu_sharded(rank, world, port, work):
    """Two ranks on one GPU: shard the documents, gather over gloo (host
    tensors), merge on rank 0; rank 0 writes its runs for comparison."""
    import cmsbwt
    import cmsbwt.dist as cdist
    dist = _init(rank, world, port)
    cfg = json.load(open(os.path.join(work, "cfg.json")))
    eng = cmsbwt.Engine(0)
    eng.initialize_reference(cfg["ref"])
    docs = cfg["docs"]
    b, e = cdist.shard_range(len(docs), world, rank)
    eng.load_collection([bytes.fromhex(d) for d in docs[b:e]])
    for _ in range(2):  # twice: the second step reuses imported state correctly
        cdist.gather_step(eng, "cpu", rle=True)
    if rank == 0:
        open(os.path.join(work, "runs.bin"), "wb").write(eng.runs_bytes())
    eng.close()
    dist.destroy_process_group()


def gpu_gather_device(rank, world, port, work):
    """gather_step on device tensors over RCCL (the bench's CMSBWT_DIST=gather
    path): the reduce, the root's slice copy and the receives run on torch's
    stream while the engine reads from its own, so gather_walk must wait for
    them.  One rank (RCCL allows one rank per GPU); rank 0 writes its runs."""
    import cmsbwt
    import cmsbwt.dist as cdist
    dist = _init(rank, world, port, backend="nccl")
    cfg = json.load(open(os.path.join(work, "cfg.json")))
    eng = cmsbwt.Engine(0)
    eng.initialize_reference(cfg["ref"])
    docs = cfg["docs"]
    b, e = cdist.shard_range(len(docs), world, rank)
    eng.load_collection([bytes.fromhex(d) for d in docs[b:e]])
    for it in range(cfg.get("steps", 1)):
        cdist.gather_step(eng, "cuda:0", rle=cfg["rle"])
        if rank == 0:
            open(os.path.join(work, f"runs{it}.bin"), "wb").write(eng.runs_bytes())
    eng.close()
    dist.destroy_process_group()


def cpu_transport(rank, world, port, work):
    """The sharded merge's exchange primitives on host tensors: uneven
    all-to-all (records of several words, empty splits), count exchange,
    all-reduce and all-gather, checked against their definitions."""
    import torch
    import cmsbwt.dist as cdist
    dist = _init(rank, world, port)
    x = cdist.Transport("cpu")
    assert (x.world, x.rank, x.staged) == (world, rank, False)
    # rank r sends (r + d) % 3 records of 5 words to rank d; record = (r, d, k, r*d, -1)
    send_counts = [(rank + d) % 3 for d in range(world)]
    rows = [[rank, d, k, rank * d, -1] for d in range(world) for k in range(send_counts[d])]
    send = torch.tensor(rows, dtype=torch.int32).reshape(-1, 5)
    recv_counts = x.counts(send_counts)
    assert recv_counts == [(s + rank) % 3 for s in range(world)]
    got = x.a2a(send, send_counts, recv_counts)
    want = [[s, rank, k, s * rank, -1] for s in range(world) for k in range(recv_counts[s])]
    assert got.tolist() == want
    # gather-to-rank-0 pattern of the run streams (uint8 and int64)
    n = 3 + rank
    sc = [n if d == 0 else 0 for d in range(world)]
    counts = [v[0] for v in x.allgather_ints([n])]
    rc = counts if rank == 0 else [0] * world
    g8 = x.a2a(torch.full((n,), 7 + rank, dtype=torch.uint8), sc, rc)
    g64 = x.a2a(torch.full((n,), (1 << 40) + rank, dtype=torch.int64), sc, rc)
    if rank == 0:
        assert g8.tolist() == [7 + r for r in range(world) for _ in range(3 + r)]
        assert g64.tolist() == [(1 << 40) + r for r in range(world) for _ in range(3 + r)]
    # all-reduce sum / max
    t = torch.arange(6, dtype=torch.int64) * (rank + 1)
    x.allreduce(t, "sum")
    assert t.tolist() == [k * world * (world + 1) // 2 for k in range(6)]
    u = torch.tensor([rank, 5 - rank], dtype=torch.uint8)
    x.allreduce(u, "max")
    assert u.tolist() == [world - 1, 5]
    if rank == 0:
        open(os.path.join(work, "ok"), "w").write("ok")
    dist.destroy_process_group()


def gpu_position_sharded(rank, world, port, work):
    """Ranks sharing one GPU run the position-sharded merge over gloo (device
    tensors staged through host memory); rank 0 writes its runs."""
    import cmsbwt
    import cmsbwt.dist as cdist
    dist = _init(rank, world, port)
    cfg = json.load(open(os.path.join(work, "cfg.json")))
    eng = cmsbwt.Engine(0)
    eng.initialize_reference(cfg["ref"])
    docs = cfg["docs"]
    b, e = cdist.shard_range(len(docs), world, rank)
    eng.load_collection([bytes.fromhex(d) for d in docs[b:e]])
    x = cdist.Transport("cuda:0")
    for it in range(cfg.get("steps", 1)):
        cdist.sharded_step(eng, "cuda:0", rle=cfg["rle"], xfer=x)
        if rank == 0:
            open(os.path.join(work, f"runs{it}.bin"), "wb").write(eng.runs_bytes())
            json.dump(eng.stats().as_dict(), open(os.path.join(work, "stats.json"), "w"))
    eng.close()
    dist.destroy_process_group()


def gpu_sharded_files(rank, world, port, work):
    """Ranks sharing one GPU: each loads its byte range of the collection file
    (cmsbwt_load_collection_file_range) and the sharded step runs over gloo;
    rank 0 writes its runs and statistics."""
    import cmsbwt
    import cmsbwt.dist as cdist
    dist = _init(rank, world, port)
    cfg = json.load(open(os.path.join(work, "cfg.json")))
    eng = cmsbwt.Engine(0)
    eng.initialize_reference(cfg["ref"])
    eng.load_collection_file_range(cfg["coll"], rank, world)
    x = cdist.Transport("cuda:0")
    cdist.sharded_step(eng, "cuda:0", rle=cfg["rle"], xfer=x)
    if rank == 0:
        if cfg.get("out"):  # the output file itself (plain .bwt expanded on the device)
            eng.write_output(cfg["out"], rle=cfg["rle"])
        else:
            open(os.path.join(work, "runs0.bin"), "wb").write(eng.runs_bytes())
        json.dump(eng.stats().as_dict(), open(os.path.join(work, "stats.json"), "w"))
    eng.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    fn, rank, world, port, work = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    globals()[fn](rank, world, port, work)
