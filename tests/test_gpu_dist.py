"""GPU: the sharded pipeline (2 ranks on one device, gloo over host memory)
produces the same .rl_bwt as one rank and as the oracle."""
import json
import os

import pytest

import cases
from test_multirank import spawn

pytestmark = pytest.mark.gpu


def test_two_rank_sharded_run_matches_oracle(oracle, tmp_path):
    rng = cases._rng(31)
    ref = cases.rand_dna(rng, 40000)
    seqs = [cases.mutate(rng, ref, 0.003) for _ in range(7)]
    work = str(tmp_path)
    rp = os.path.join(work, "ref.fa")
    open(rp, "wb").write(cases.fasta([ref]))
    coll = cases.fasta(seqs)
    cp = os.path.join(work, "coll.fa")
    open(cp, "wb").write(coll)
    assert oracle.run(rp, cp, os.path.join(work, "o"), rle=True)[0] == 0
    docs, _ = cases.py_read_docs(coll)
    json.dump({"ref": rp, "docs": [d.hex() for d in docs]}, open(os.path.join(work, "cfg.json"), "w"))
    spawn("gpu_sharded", 2, work)
    assert open(os.path.join(work, "runs.bin"), "rb").read() == open(os.path.join(work, "o.rl_bwt"), "rb").read()
