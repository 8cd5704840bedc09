"""CPU, world_size 2 (gloo): document sharding + gather-to-merge-rank.

The walk and j-scan are document-local, so running the oracle
on each contiguous shard of documents must reproduce the slices of the global
head arrays, and the shards' per-position counts must sum to the global ones.
The gloo run exercises cmsbwt.dist.gather_walk exactly as bench.py does."""
import json
import os
import socket
import subprocess
import sys

import pytest

import cases

HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn(fn, world, work, timeout=240):
    port = _port()
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), fn, str(r), str(world),
                               str(port), work]) for r in range(world)]
    rcs = [p.wait(timeout=timeout) for p in procs]
    assert rcs == [0] * world, rcs


def test_gather_walk_gloo_two_ranks(oracle, tmp_path):
    rng = cases._rng(21)
    ref = cases.rand_dna(rng, 6000)
    seqs = [cases.mutate(rng, ref, 0.01) for _ in range(5)]
    work = str(tmp_path)
    rp = os.path.join(work, "ref.fa")
    open(rp, "wb").write(cases.fasta([ref]))
    # global: leading '>' gives an empty first document (6 documents)
    gp = os.path.join(work, "global.fa")
    open(gp, "wb").write(cases.fasta(seqs))
    assert oracle.run(rp, gp, os.path.join(work, "g"), dump_dir=os.path.join(work, "global"))[0] == 0
    # shard 0: [empty, s0, s1]; shard 1 (headerless start): [s2, s3, s4]
    s0 = cases.fasta(seqs[:2])
    s1 = seqs[2] + b"\n" + cases.fasta(seqs[3:])
    ndocs, chars = [], []
    for r, content in enumerate((s0, s1)):
        p = os.path.join(work, f"s{r}.fa")
        open(p, "wb").write(content)
        docs, _ = cases.py_read_docs(content)
        ndocs.append(len(docs))
        chars.append(sum(len(d) for d in docs))
        assert oracle.run(rp, p, os.path.join(work, f"o{r}"), dump_dir=os.path.join(work, f"shard{r}"))[0] == 0
    assert ndocs == [3, 3]
    json.dump({"ndocs": ndocs, "chars": chars}, open(os.path.join(work, "cfg.json"), "w"))
    spawn("cpu_gather", 2, work)
    assert os.path.exists(os.path.join(work, "ok"))


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_range_partitions(world):
    import cmsbwt.dist as cdist
    for total in (0, 1, 7, 1000, 1001):
        rs = [cdist.shard_range(total, world, r) for r in range(world)]
        assert rs[0][0] == 0 and rs[-1][1] == total
        assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
        assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_merge_transport_gloo(tmp_path, world):
    """The exchange primitives of the position-sharded merge (cmsbwt.dist.Transport)."""
    spawn("cpu_transport", world, str(tmp_path))
    assert os.path.exists(os.path.join(str(tmp_path), "ok"))
