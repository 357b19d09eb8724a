"""Multi-process RCCL runs of the sharded engines: one process per GPU, as bench.py
runs them at N > 1.  Needs at least two visible devices (the
driver's 8-GPU node); on a one-GPU box every test here skips.

* dense (config 5's engine, csrc/dist_sub.hip): per-axis split communicators, halo
  messages as ncclSend / ncclRecv on the exchange streams;
* sparse (configs 3/4, csrc/dist_sparse.hip): the reference's LOOK_UP / RESOLVE p2p pair
  (src/new_process.py:159,186) batched per tier as ncclGroup send / recv.

Every rank's table digest is summed and compared with the C oracle's (committed in
tests/golden/oracle_digests.json, or computed here for 6 heaps).
"""
import json
import multiprocessing as mp
import os

import numpy as np
import pytest

from conftest import GOLDEN, digest

pytestmark = pytest.mark.gpu

SUB, TOOT, OTH = 5, 3, 4


def _devices():
    import torch   # device_count() does not initialise the GPU in this process
    return torch.cuda.device_count()


def _rank_main(rank, world, game, params, opts, uidq, out):
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")   # as bench.py: a queue per stream
    try:
        import ctypes
        from gamesmanmpi_amd import Context, _lib
        ctx = Context(game, params, device=rank)
        if rank == 0:
            buf = ctypes.create_string_buffer(128)
            _lib.check(_lib.lib().gm_comm_unique_id(buf, 128))
            for _ in range(world - 1):
                uidq.put(buf.raw)
            uid = buf.raw
        else:
            uid = uidq.get(timeout=120)
        ctx.set_comm(rank, world, uid)
        for k, v in opts.items():
            ctx.set_option(getattr(_lib, "OPT_" + k.upper()), v)
        n, rec = ctx.solve(ctx.initial())
        d, m = ctx.digest()
        out.put({"rank": rank, "n": n, "rec": rec, "digest": d, "m": m,
                 "tiers": [int(x) for x in ctx.tier_counts()], "exchanged": ctx.stats()["exchanged_bytes"]})
        ctx.close()
    except Exception as e:  # reported to the parent
        out.put({"rank": rank, "error": repr(e)})


def _run(world, game, params, opts=None):
    if _devices() < world:
        pytest.skip("needs %d GPUs (one process per GPU over RCCL)" % world)
    ctx = mp.get_context("spawn")
    uidq, out = ctx.Queue(), ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, world, game, params, opts or {}, uidq, out))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [out.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all("error" not in r for r in res), res
    return sorted(res, key=lambda r: r["rank"])


def _summed(res):
    return sum(r["digest"] for r in res) & ((1 << 64) - 1), sum(r["m"] for r in res)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_dense_rccl_2_32_matches_oracle_digest(world):
    """Config 5 at full size, block-owner sharded over `world` processes."""
    ref = json.load(open(os.path.join(GOLDEN, "oracle_digests.json")))["subtract_8"]
    res = _run(world, SUB, (8,))
    assert all(r["n"] == 1 << 32 and r["rec"] == ref["root_record"] for r in res)
    assert _summed(res) == (ref["digest"], 1 << 32)
    assert sum(r["exchanged"] for r in res) > 0


@pytest.mark.parametrize("owner", [0, 1])
def test_dense_rccl_6_heaps_vs_oracle(oracle, owner):
    ref = oracle.subtract_dense(6)
    keys = np.arange(1 << 24, dtype=np.uint64)
    res = _run(2, SUB, (6,), {"dist_owner": owner})
    assert _summed(res) == (digest(keys, ref), 1 << 24)


@pytest.mark.parametrize("world", [2, 8])
@pytest.mark.parametrize("name,game,params", [("othello_4x4", OTH, (4, 4)), ("toot_6x4", TOOT, (6, 4))])
def test_sparse_rccl_matches_oracle_digest(world, name, game, params):
    ref = json.load(open(os.path.join(GOLDEN, "oracle_digests.json")))[name]
    res = _run(world, game, params)
    assert all(r["n"] == ref["positions"] and r["rec"] == ref["root_record"] for r in res)
    assert _summed(res) == (ref["digest"], ref["positions"])
    if "per_ply" in ref:
        assert all(r["tiers"] == ref["per_ply"] for r in res)
