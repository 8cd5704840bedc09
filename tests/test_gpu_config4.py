"""GPU: BASELINE config 4 -- the headline workload (10 MB reference + 1000
copies @0.1 % SNP, 10 GB, -r) sharded over N ranks -- run through bench.py's
own N > 1 path.

The driver launches `bench.py --gpus N` under torchrun with one rank per GPU
over RCCL.  Here the ranks share the test GPU (CMSBWT_BENCH_SAME_GPU=1: every
rank on device 0, gloo with host staging instead of RCCL, which allows one rank
per device); the sharding, the sharded merge (dist_merge.hip) and every
collective are the ones the N-GPU run issues.  Rank 0's runs of the timed step
must equal the oracle's golden for this exact workload (golden synth_c3:
sha256 of the .rl_bwt, headNumber, keys, Rank, runs and the three counter
totals), FN:1138-1352 (document loop, sharded) and FN:1387-1777 (merge)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_bench(world, extra=(), env_extra=None, timeout=900):
    env = dict(os.environ, CMSBWT_BENCH_SAME_GPU="1", CMSBWT_BENCH_REHEARSAL="1", PYTHONUNBUFFERED="1")
    env.update(env_extra or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--steps", "1", "--warmup", "0", "--no-cpu", "--no-e2e", *extra]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("world", [2, 4, 8])
def test_config4_sharded_bench_golden(world):
    out = run_bench(world)
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))["synth_c3"]
    par = out["parity"]
    assert par["verdict"] == "bit-exact vs oracle golden", par
    assert par["heads"] == g["headNumber"] == 100572666
    assert par["rank"] == g["Rank"] == 54555418
    assert (par["counter_bad"], par["counter_good"], par["counter_nothing"]) == \
        (g["counterBad"], g["counterGood"], g["counterDoNothing"])
    # a rehearsal: the ranks share device 0, and the line says so
    assert out["n_gpus"] == 1 and out["ranks"] == world and "rehearsal" in out
    assert len(out["per_rank"]) == world
    # every rank walked its share of the documents; the merge stage is timed
    assert sum(r["chars"] for r in out["per_rank"]) == 10**10
    assert sum(r["heads"] for r in out["per_rank"]) == g["headNumber"]
    assert out["stages_ms"]["merge"] > 0 and out["stages_ms"]["ms_walk"] > 0
    print(json.dumps({"world": world, "ms_per_step": out["ms_per_step"], "stages_ms": out["stages_ms"],
                      "per_rank": out["per_rank"], "hbm_peak_gib": out["hbm_peak_gib"]}))


def run_bench_in_process(world, extra=(), env_extra=None, timeout=900):
    """bench.py --gpus N without a launcher: the product's in-process rank
    group (multi.hip, one host thread + context per rank; on a one-GPU box
    every rank on device 0, PEER transport as device-local copies)."""
    env = dict(os.environ, PYTHONUNBUFFERED="1", CMSBWT_BENCH_REHEARSAL="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    env.update(env_extra or {})
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--steps", "2", "--warmup", "1",
           "--no-cpu", "--no-e2e", *extra]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("world", [2, 4])
def test_config4_in_process_bench_golden(world):
    """`bench.py --gpus N` (rehearsal on a box with fewer devices) reports
    n_gpus = the distinct devices, ranks = N, per-rank rows, and rank 0's runs
    of the timed step equal the golden (FN:1387-1777 sharded)."""
    out = run_bench_in_process(world)
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))["synth_c3"]
    par = out["parity"]
    assert par["verdict"] == "bit-exact vs oracle golden", par
    assert par["heads"] == g["headNumber"] and par["rank"] == g["Rank"]
    assert (par["counter_bad"], par["counter_good"], par["counter_nothing"]) == \
        (g["counterBad"], g["counterGood"], g["counterDoNothing"])
    import torch
    ndev = torch.cuda.device_count()
    assert out["ranks"] == world and len(out["per_rank"]) == world
    assert len(out["per_rank_devices"]) == world
    assert out["n_gpus"] == len(set(out["per_rank_devices"])) == min(world, ndev)
    assert ("rehearsal" in out) == (world > ndev)
    assert sum(r["chars"] for r in out["per_rank"]) == 10**10
    assert sum(r["heads"] for r in out["per_rank"]) == g["headNumber"]
    print(json.dumps({"world": world, "ms_per_step": out["ms_per_step"], "stages_ms": out["stages_ms"],
                      "per_rank": out["per_rank"]}))


def test_bench_refuses_shared_devices():
    """More in-process ranks than devices (or torchrun ranks on one device)
    without CMSBWT_BENCH_REHEARSAL=1: exit 2 and no number."""
    import torch
    ndev = torch.cuda.device_count()
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "CMSBWT_BENCH_REHEARSAL", "CMSBWT_BENCH_SAME_GPU"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(ndev + 1), "--steps", "1", "--warmup", "0",
           "--no-cpu", "--no-e2e"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, (r.returncode, r.stdout[-500:], r.stderr[-1500:])
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1 and "error" in json.loads(lines[0]) and "value" not in json.loads(lines[0])
    env2 = dict(env, CMSBWT_BENCH_SAME_GPU="1", WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run(cmd[:3] + ["2"] + cmd[4:], cwd=ROOT, env=env2, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, (r.returncode, r.stdout[-500:], r.stderr[-1500:])
