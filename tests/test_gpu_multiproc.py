"""Multi-process runs of the sharded engines: one process per rank, as bench.py runs them at
N > 1.  The RCCL tests need one visible device per rank (the driver's
8-GPU node) and skip on a one-GPU box; the box engine's IPC-transport tests run there too,
their ranks sharing the GPU (RCCL refuses two ranks on one device).

* dense, 8 heaps (config 5's engine, csrc/dist_box.hip): every box on one rank, per-axis
  split communicators, each batch's halo boxes as ncclSend / ncclRecv on the exchange
  streams;
* dense, block engine (other heap counts, or GM_OPT_SUB_INTERLEAVE 10; csrc/dist_sub.hip):
  per-axis split communicators, halo messages as ncclSend / ncclRecv on the exchange streams;
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


def _rank_main(rank, world, phase, game, params, opts):
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")   # as bench.py: a queue per stream
    import ctypes
    import torch.distributed as tdist
    from gamesmanmpi_amd import Context, _lib
    tdist.init_process_group("gloo", rank=rank, world_size=world)   # MASTER_* from the parent
    opts = dict(opts)
    shared = opts.pop("share_gpus", False)   # ranks round-robin over the visible GPUs (IPC transport)
    ctx = Context(game, params, device=rank % _lib.lib().gm_device_count() if shared else rank)
    phase("unique id")
    uid = [None]
    if rank == 0:
        buf = ctypes.create_string_buffer(128)
        _lib.check(_lib.lib().gm_comm_unique_id(buf, 128))
        uid[0] = buf.raw
    tdist.broadcast_object_list(uid, src=0)
    phase("communicator")
    ctx.set_comm(rank, world, uid[0])
    root = opts.pop("root", None)
    qkeys = opts.pop("query_keys", None)
    want_export = opts.pop("export", False)
    solves = opts.pop("solves", 1)
    for k, v in opts.items():
        ctx.set_option(getattr(_lib, "OPT_" + k.upper()), v)
    digests = []
    for i in range(solves):
        phase("solve %d" % i)
        n, rec = ctx.solve(ctx.initial() if root is None else root)
        phase("digest %d" % i)
        digests.append(ctx.digest())
    d, m = digests[-1]
    res = {"rank": rank, "n": n, "rec": rec, "digest": d, "m": m, "digests": digests,
           "tiers": [int(x) for x in ctx.tier_counts()], "exchanged": ctx.stats()["exchanged_bytes"]}
    if qkeys is not None:
        res["query"] = [int(x) for x in ctx.query(np.array(qkeys, dtype=np.uint64))]
    if want_export:
        k, r = ctx.export()
        res["export"] = (k.tolist(), r.tolist())
    ctx.close()
    return res


def _run(world, game, params, opts=None, shared=False):
    """Every rank in its own process; on a timeout, an error or a dead rank, every
    rank is terminated then killed and the failure names each rank's last phase
    (tests/mp_ranks.py).  shared: the ranks may share GPUs (the box engine's IPC transport)."""
    if shared:
        if _devices() < 1:
            pytest.skip("needs a GPU")
        opts = dict(opts or {}, share_gpus=True)
    elif _devices() < world:
        pytest.skip("needs %d GPUs (one process per GPU over RCCL)" % world)
    import socket
    from mp_ranks import run_ranks
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    return run_ranks(_rank_main, world, (game, params, opts or {}), timeout=240)


def _summed(res):
    return sum(r["digest"] for r in res) & ((1 << 64) - 1), sum(r["m"] for r in res)


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("interleave", [20, 10])
def test_dense_rccl_2_32_matches_oracle_digest(world, interleave):
    """Config 5 at full size over `world` processes: the box engine (20, the default) and the
    block engine (10), both with halo messages over RCCL."""
    ref = json.load(open(os.path.join(GOLDEN, "oracle_digests.json")))["subtract_8"]
    res = _run(world, SUB, (8,), {"sub_interleave": interleave})
    assert all(r["n"] == 1 << 32 and r["rec"] == ref["root_record"] for r in res)
    assert _summed(res) == (ref["digest"], 1 << 32)
    assert sum(r["exchanged"] for r in res) > 0


@pytest.mark.parametrize("sym", [0, 1])
def test_box_rccl_custom_root_vs_oracle(oracle, sym):
    """The split box engine over 2 processes at a custom root, with and without the symmetric
    fill: the summed digests equal the oracle's, and gm_query on a rank answers exactly the
    keys of the boxes it computed (0xFFFF for the others: include/gmsolve.h gm_query), so
    every sampled key is answered by one rank, with the oracle's record."""
    from gamesmanmpi_amd import _lib
    root = 0x33557777
    ok, orec = oracle.solve(SUB, (8,), root=root)
    sample = ok[:: max(1, len(ok) // 4000)]
    want = orec[:: max(1, len(ok) // 4000)]
    res = _run(2, SUB, (8,), {"dist_symmetry": sym, "root": root, "query_keys": sample.tolist()})
    assert _summed(res) == (digest(ok, orec), len(ok))
    q = np.array([r["query"] for r in res])
    answered = q != _lib.REC_UNSOLVED
    assert (answered.sum(axis=0) == 1).all()
    assert np.array_equal(np.where(answered, q, 0).sum(axis=0), want)


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


def _oracle_box(oracle, root):
    ok, orec = oracle.solve(SUB, (8,), root=root)
    return ok, orec, (digest(ok, orec), len(ok))


@pytest.mark.parametrize("world,root,batch,sym", [(2, 0x33557777, 1, 1), (3, 0x33557777, 2, 0),
                                                  (4, 0x23457777, 1, 1)])
def test_box_ipc_ranks_vs_oracle(oracle, world, root, batch, sym):
    """The split box engine across PROCESSES with the IPC transport (GM_OPT_BOX_TRANSPORT 1):
    each process one rank, the halo messages peer-copied into the receiver's buffer mapped
    through hipIpcOpenMemHandle, completion flags set and polled by stream-ordered kernels --
    runs on a one-GPU box, the ranks sharing the GPU (RCCL refuses that).  Three solves in a
    row (the flags' sequence numbers and the back-pressure on reused buffers): the summed
    digests equal the C oracle's every time, every rank reports the root record, and every
    sampled key is answered by exactly one rank (gm_query).  GM_OPT_POISON 1: every received
    box goes back to 0xFF after it is read, so solves 2 and 3 read nothing solve 1 left."""
    from gamesmanmpi_amd import _lib
    ok, orec, want = _oracle_box(oracle, root)
    sample = ok[:: max(1, len(ok) // 3000)]
    res = _run(world, SUB, (8,), {"box_transport": 1, "root": root, "dist_batch": batch, "dist_symmetry": sym,
                                  "solves": 3, "poison": 1, "query_keys": sample.tolist()}, shared=True)
    for i in range(3):
        assert (sum(r["digests"][i][0] for r in res) & ((1 << 64) - 1), sum(r["digests"][i][1] for r in res)) == want
    rec = orec[np.searchsorted(ok, root)]
    assert all(r["rec"] == rec for r in res)
    q = np.array([r["query"] for r in res])
    answered = q != _lib.REC_UNSOLVED
    assert (answered.sum(axis=0) == 1).all()
    assert np.array_equal(np.where(answered, q, 0).sum(axis=0), orec[:: max(1, len(ok) // 3000)])
    assert sum(r["exchanged"] for r in res) > 0


def test_box_ipc_ranks_2_32_matches_oracle_digest():
    """Config 5 at full size over 4 processes with the IPC transport (sharing one GPU on a
    one-GPU box): the summed digests equal the committed oracle digest, twice."""
    ref = json.load(open(os.path.join(GOLDEN, "oracle_digests.json")))["subtract_8"]
    res = _run(4, SUB, (8,), {"box_transport": 1, "dist_batch": 1, "solves": 2, "poison": 1}, shared=True)
    for i in range(2):
        assert (sum(r["digests"][i][0] for r in res) & ((1 << 64) - 1),
                sum(r["digests"][i][1] for r in res)) == (ref["digest"], 1 << 32)
    assert all(r["n"] == 1 << 32 and r["rec"] == ref["root_record"] for r in res)


@pytest.mark.parametrize("world", [2, 4])
def test_box_ipc_dataflow_ranks_vs_oracle(oracle, world):
    """The split dataflow across processes (GM_OPT_BOX_FLOW 1 + GM_OPT_BOX_TRANSPORT 1): each
    process's chain one launch, its halo boxes and their flags stored into the receiving
    process's table and flag array through the IPC mappings -- a box of one process waits on a
    flag another process stores.  The ranks share the GPU here, so each launch takes its share
    of the resident workgroups.  Three solves: the summed digests equal the oracle's."""
    root = 0x33557777
    ok, orec, want = _oracle_box(oracle, root)
    res = _run(world, SUB, (8,), {"box_transport": 1, "box_flow": 1, "root": root, "solves": 3, "poison": 1},
               shared=True)
    for i in range(3):
        assert (sum(r["digests"][i][0] for r in res) & ((1 << 64) - 1), sum(r["digests"][i][1] for r in res)) == want


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("name,game,params", [("othello_4x4", OTH, (4, 4)), ("toot_4x4", TOOT, (4, 4))])
def test_sparse_ipc_ranks_vs_oracle_digest(world, name, game, params):
    """the hash-sharded sparse engine (csrc/dist_sparse.hip, north_star's
    partition for configs 3/4) across PROCESSES, one rank each, with the IPC transport
    (GM_OPT_SPARSE_TRANSPORT 1): every tier's LOOK_UP keys and RESOLVE scores are pulled out of
    the owners' send buffers through HIP IPC mappings, counts / totals / the root record
    all-gathered through the shared-memory segment.  Runs on a one-GPU box, the ranks sharing
    the GPU.  Receive buffers are poisoned with 0xFF before every exchange (GM_OPT_POISON 1), and
    two solves run back to back: the summed digests, the per-tier counts and the root record
    equal the committed oracle's both times (reference src/new_process.py:156-160, :179-187)."""
    ref = json.load(open(os.path.join(GOLDEN, "oracle_digests.json")))[name]
    res = _run(world, game, params, {"sparse_transport": 1, "poison": 1, "solves": 2}, shared=True)
    for i in range(2):
        assert (sum(r["digests"][i][0] for r in res) & ((1 << 64) - 1),
                sum(r["digests"][i][1] for r in res)) == (ref["digest"], ref["positions"])
    assert all(r["n"] == ref["positions"] and r["rec"] == ref["root_record"] for r in res)
    per = ref.get("per_ply") or ref.get("per_tier")
    assert all(r["tiers"] == per for r in res)
    assert all(r["exchanged"] > 0 for r in res)


def test_sparse_ipc_ranks_toot_5x4_vs_oracle_digest():
    """Toot 5x4 (70,184,763 positions) over 3 processes with the IPC transport: larger tiers,
    so the send buffers grow and come back from the allocation cache between exchanges (each
    peer allocation is mapped once per solve); summed digests, per-ply counts and the root
    record equal the committed oracle's."""
    ref = json.load(open(os.path.join(GOLDEN, "oracle_digests.json")))["toot_5x4"]
    res = _run(3, TOOT, (5, 4), {"sparse_transport": 1}, shared=True)
    assert _summed(res) == (ref["digest"], ref["positions"])
    assert all(r["n"] == ref["positions"] and r["rec"] == ref["root_record"] for r in res)
    assert all(r["tiers"] == ref["per_ply"] for r in res)


def test_sparse_ipc_ranks_query_othello_golden():
    """Othello 4x4 over 3 processes (IPC transport): every key of the reference plugin's golden
    table is answered by exactly one rank (its hash owner), with the golden record."""
    from gamesmanmpi_amd import _lib
    g = np.load(os.path.join(GOLDEN, "othello_4x4.npz"))
    res = _run(3, OTH, (4, 4), {"sparse_transport": 1, "query_keys": g["keys"].tolist()}, shared=True)
    q = np.array([r["query"] for r in res])
    answered = q != _lib.REC_UNSOLVED
    assert (answered.sum(axis=0) == 1).all()
    assert np.array_equal(np.where(answered, q, 0).sum(axis=0), g["records"])


@pytest.mark.parametrize("poison,caught", [(2, True), (3, False)])
def test_box_ipc_early_read_caught_by_poison(oracle, poison, caught):
    """a fault injected into the IPC transport must fail solve 2, not only
    solve 1.  Test hook GM_OPT_POISON 2 / 3: from solve 2 on, rank 1 reads its halo boxes
    without waiting for their arrival flags (as if the flags were set early) while rank 0, the
    sender, is held 50 ms at the start of its solve.  With the received boxes poisoned (2), the
    early reads see 0xFF and solve 2's summed digest differs from the oracle's; solve 1 is
    exact.  Without poisoning (3) the same fault is invisible -- the early reads find solve 1's
    identical codes -- which is why the tests and the bench's probe poison."""
    root = 0x33557777
    ok, orec, want = _oracle_box(oracle, root)
    res = _run(2, SUB, (8,), {"box_transport": 1, "root": root, "dist_batch": 1, "solves": 3, "poison": poison},
               shared=True)
    got = [(sum(r["digests"][i][0] for r in res) & ((1 << 64) - 1), sum(r["digests"][i][1] for r in res))
           for i in range(3)]
    assert got[0] == want
    if caught:
        assert got[1] != want and got[2] != want
    else:
        assert got[1] == want and got[2] == want


@pytest.mark.parametrize("world", [2, 3])
def test_othello8_ipc_ranks_vs_reference_golden(world):
    """Othello 8x8 (128-bit keys) from the 10-empty endgame root across PROCESSES with the IPC
    transport, the ranks sharing the GPU: the ranks' exports partition the solved set, and
    every record equals the reference plugin's golden table."""
    import hashlib
    from conftest import golden
    from gamesmanmpi_amd import _lib, games
    codec = games.OthelloCodec(8, 8)
    root = codec.key(bytes.fromhex("303800204018057a4646bfdebfe6fa800200").decode("latin-1"))
    res = _run(world, OTH, (8, 8), {"sparse_transport": 1, "poison": 1, "root": root, "export": True}, shared=True)
    got = {}
    for r in res:
        for w, rec in zip(*r["export"]):
            pos = codec.pos(_lib.words_to_int(w))
            h = int.from_bytes(hashlib.blake2b(pos.encode("ISO-8859-1"), digest_size=8).digest(), "big")
            assert h not in got
            got[h] = rec
    keys, recs = golden("othello_8x8_endgame")
    assert got == dict(zip(keys.tolist(), recs.tolist()))
    assert all(r["n"] == 56552 for r in res)
