"""The multi-GPU dense path's schedule, checked on the CPU (no GPU needed).

Each rank's plan -- block-owner partition, halo lists, op list -- comes from the
product through gm_dist_plan (the host code gm_solve runs; csrc/dist_sub.hip).
tests/dist_sim.py executes the RCCL-mode op lists of all ranks under HIP stream /
event and RCCL point-to-point semantics in random interleavings, and, over
torch.distributed gloo with one process per rank, moves the halos as real
messages carrying the C oracle's values.  The GPU side of the same schedule is
tests/test_gpu_sharded.py (loopback ranks on one device).
"""
import multiprocessing as mp
import socket

import numpy as np
import pytest

import dist_sim as S
from gamesmanmpi_amd import _lib, GMError


def plans(heaps, world, batch=4, slots=4, symmetry=1, owner=0):
    return [S.load_plan(heaps, world, r, batch, slots, symmetry, owner) for r in range(world)]


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("batch,slots,symmetry", [(4, 4, 1), (4, 4, 0), (1, 1, 1), (1, 1, 0), (2, 1, 1),
                                                  (3, 2, 0), (100, 2, 1)])
def test_schedule_is_deadlock_free_and_race_free(world, batch, slots, symmetry):
    P = plans(6, world, batch, slots, symmetry)
    for seed in range(3):
        assert S.simulate(P, seed=seed)


def test_schedule_full_size_8_ranks():
    """The bench configuration: 2^32 positions, 8 ranks, default batch / ring / fill."""
    P = plans(8, 8)
    shape = P[0]
    assert (shape["low"], shape["high"], shape["ntiers"], shape["nbatch"], shape["g"]) == (3, 5, 76, 19, 3)
    assert S.simulate(P, seed=1)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_partition_and_halo_volume(world):
    """Every block has one owner, ranks own equal shares, and the symmetric fill cuts the
    halo that crosses a link to 1/16, 1/8, 1/4 of the split-heap layers."""
    heaps = 8
    g = world.bit_length() - 1
    sent = {}
    for sym in (0, 1):
        total = 0
        owned = np.zeros(1 << 20, dtype=np.int64)
        for r in range(world):
            _, own = _lib.dist_plan(heaps, world, r, _lib.PLAN_OWN, symmetry=sym)
            owned[own] += 1
            assert len(own) == (1 << 20) // world
            for a in range(g):
                total += len(_lib.dist_plan(heaps, world, r, _lib.PLAN_SEND, axis=a, symmetry=sym)[1])
        assert (owned == 1).all()
        sent[sym] = total * 4096
    assert sent[0] == g * (512 << 20)           # 2 of 16 layers of the 4 GiB table per split heap
    assert sent[1] == {2: 32, 4: 128, 8: 384}[world] << 20


@pytest.mark.parametrize("owner", [0, 1])
@pytest.mark.parametrize("world", [2, 4, 8])
def test_tier_kernel_destinations_match_the_lists(world, owner):
    """GM_PLAN_XDEST (what the tier kernel writes besides each own block) is exactly the
    symmetric-fill images and the halo ring slots of the plan's fill and send lists."""
    for r in range(world):
        p = S.load_plan(7, world, r, owner=owner)
        want = {}
        for dst, src in p["fill"].reshape(-1, 2).tolist():
            want.setdefault(src, set()).add((0, dst))
        for a in range(p["g"]):
            off, blocks = p["send"][a]
            for j in range(len(off) - 1):
                for k, H in enumerate(blocks[off[j]:off[j + 1]].tolist()):
                    want.setdefault(H, set()).add((1 + a, j << 16 | k))
        got = {}
        xoff, xd = p["xoff"], p["xd"].reshape(-1, 2)
        assert len(xoff) == len(p["own"]) + 1
        for i, H in enumerate(p["own"].tolist()):
            d = {tuple(v) for v in xd[xoff[i]:xoff[i + 1]].tolist()}
            if d:
                got[H] = d
        assert got == want
        assert sum(len(v) for v in want.values()) == len(xd)


@pytest.mark.parametrize("heaps,world", [(6, 2), (6, 4), (7, 4), (7, 8)])
@pytest.mark.parametrize("batch,slots", [(4, 4), (1, 1), (2, 1), (100, 2)])
def test_tier_balanced_schedule_is_deadlock_free_and_race_free(heaps, world, batch, slots):
    """GM_OPT_DIST_OWNER 1: the same checks on the tier-balanced partition (its halo is
    the tie blocks and whatever no heap permutation maps onto the receiver)."""
    P = plans(heaps, world, batch, slots, owner=1)
    for seed in range(2):
        assert S.simulate(P, seed=seed)


def test_tier_balanced_full_size_8_ranks():
    P = plans(8, 8, owner=1)
    assert S.simulate(P, seed=1)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_tier_balanced_partition(world):
    """Owner 1 at 2^32: every block has one owner; summed over tiers, the largest rank
    share of a tier (the tier chain's critical path) drops against owner 0; the
    halo that crosses a link is the blocks no heap permutation can fill."""
    heaps, g = 8, world.bit_length() - 1
    crit, sent = {}, {}
    for owner in (0, 1):
        owned = np.zeros(1 << 20, dtype=np.int64)
        per_tier, total = [], 0
        for r in range(world):
            off, own = _lib.dist_plan(heaps, world, r, _lib.PLAN_OWN, owner=owner)
            owned[own] += 1
            per_tier.append(np.diff(off.astype(np.int64)))
            for a in range(g):
                total += len(_lib.dist_plan(heaps, world, r, _lib.PLAN_SEND, axis=a, owner=owner)[1])
        assert (owned == 1).all()
        crit[owner] = int(np.array(per_tier).max(0).sum())
        sent[owner] = total
    assert crit == {2: {0: 690152, 1: 557056}, 4: {0: 442952, 1: 295936}, 8: {0: 282320, 1: 193568}}[world]
    assert sent[1] == {2: 15, 4: 480, 8: 12896}[world]


def test_tier_balanced_needs_symmetric_fill():
    with pytest.raises(GMError):
        _lib.dist_plan(8, 2, 0, _lib.PLAN_OWN, symmetry=0, owner=1)


def test_plan_rejects_impossible_splits():
    with pytest.raises(GMError):
        _lib.dist_plan(5, 8, 0, _lib.PLAN_SHAPE)      # 2 block heaps cannot split 8 ways
    with pytest.raises(GMError):
        _lib.dist_plan(8, 3, 0, _lib.PLAN_SHAPE)      # world must be 2, 4 or 8
    with pytest.raises(GMError):
        _lib.dist_plan(8, 2, 2, _lib.PLAN_OWN)        # rank out of range


def _mutate(P, rank, pred, action):
    """Copy of the plans with the first op of `rank` matching pred dropped or moved."""
    Q = [dict(p) for p in P]
    ops = Q[rank]["ops"].tolist()
    i = next(k for k, o in enumerate(ops) if pred(o))
    o = ops.pop(i)
    if action == "later":
        ops.insert(min(len(ops), i + 3), o)
    Q[rank]["ops"] = np.array(ops, dtype=np.int64).reshape(-1, 6)
    return Q


@pytest.mark.parametrize("what", ["unpack_wait", "fill", "send_before_tier", "slot_wait", "recv"])
def test_simulator_catches_broken_schedules(what):
    """The checker bites: each injected schedule bug is reported."""
    P = plans(6, 4, batch=2, slots=1, symmetry=1)
    upper = 3
    if what == "unpack_wait":      # S no longer waits for the halo's unpack before its tiers
        mid = P[upper]["nbatch"] // 2  # a batch whose tiers need the halo (rank 3's blocks start at tier 16)
        Q = _mutate(P, upper, lambda o: o[0] == S.OP_WAIT and o[2] == S.EV_UNPACKED and o[3] == 0 and o[4] == mid,
                    "drop")
    elif what == "fill":           # the symmetric fill of one tier is lost
        Q = [dict(p) for p in P]
        fo = Q[upper]["fill_off"].astype(np.int64)
        t = next(t for t in range(len(fo) - 1) if fo[t + 1] > fo[t])
        Q[upper]["fill"] = np.delete(Q[upper]["fill"], np.arange(fo[t], fo[t + 1]))
        fo[t + 1:] -= fo[t + 1] - fo[t]
        Q[upper]["fill_off"] = fo
    elif what == "send_before_tier":   # the lower rank marks a message complete before its last tier
        Q = [dict(p) for p in P]
        ops = Q[0]["ops"].tolist()
        i = next(k for k, o in enumerate(ops) if o[0] == S.OP_RECORD and o[2] == S.EV_PACKED and o[3] == 0)
        ops.insert(i - 1, ops.pop(i))
        Q[0]["ops"] = np.array(ops, dtype=np.int64).reshape(-1, 6)
    elif what == "slot_wait":      # a tier writes a ring slot without waiting for its previous send
        Q = _mutate(P, 0, lambda o: o[0] == S.OP_WAIT and o[2] == S.EV_XCH and o[3] == 0 and o[1] == 1 and o[4] == 4,
                    "drop")
    else:                          # a receive is dropped: its send never matches
        Q = _mutate(P, upper, lambda o: o[0] == S.OP_RECV, "drop")
    caught = 0
    for seed in range(20):          # a race shows only in some interleavings (the seeds are fixed)
        try:
            S.simulate(Q, seed=seed)
        except S.SimError:
            caught += 1
    assert caught > 0


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,batch,slots,symmetry,owner", [(2, 4, 4, 1, 0), (2, 1, 1, 0, 0), (4, 4, 4, 1, 0),
                                                               (4, 2, 1, 0, 0), (2, 1, 1, 1, 1), (4, 4, 2, 1, 1)])
def test_gloo_ranks_exchange_halos(world, batch, slots, symmetry, owner):
    """world_size > 1 over torch.distributed gloo: every rank runs its own RCCL-mode op
    list as a host program; after the solve every own and every halo block it holds
    equals the oracle's (6 heaps, 16.7 M positions)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=S.gloo_main, args=(r, world, port, 6, batch, slots, symmetry, q, owner))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all("error" not in r for r in res), res
    assert sorted(r["rank"] for r in res) == list(range(world))
    assert all(r["own_ok"] and r["held_ok"] for r in res), res
    assert sum(r["own_blocks"] for r in res) == 1 << 12
    assert any(r["halo_blocks"] > 0 for r in res)


OP_TIER, OP_SEND, OP_RECORD, OP_WAIT = 0, 3, 5, 6
EV_XCH = 1


@pytest.mark.parametrize("owner,heaps,world", [(0, 6, 2), (0, 7, 4), (0, 8, 8), (1, 6, 2), (1, 7, 4), (1, 8, 8)])
def test_ring_slot_waits_name_the_last_nonempty_message(owner, heaps, world):
    """GM_PLAN_OPS at ONE ring slot: before the tier that starts writing halo message jj
    into its slot, the compute stream waits for the exchange of the slot's previous
    NON-EMPTY message (empty messages record nothing), and every such wait names a
    message whose exchange was recorded earlier.  Covers owner 0 and 1."""
    for batch in (1, 3):
        shape_off, shape = _lib.dist_plan(heaps, world, 0, _lib.PLAN_SHAPE, batch=batch, slots=1, owner=owner)
        g, nslots = int(shape[6]), int(shape[5])
        assert nslots == 1
        lo = shape_off[0::2].astype(int)
        for r in range(world):
            _, ops = _lib.dist_plan(heaps, world, r, _lib.PLAN_OPS, batch=batch, slots=1, owner=owner)
            ops = ops.reshape(-1, 6).astype(int)
            for a in range(g):
                if (r >> a) & 1:
                    continue   # upper side of axis a: receives only
                soff, _ = _lib.dist_plan(heaps, world, r, _lib.PLAN_SEND, axis=a, batch=batch, slots=1, owner=owner)
                nonempty = [j for j in range(len(soff) - 1) if soff[j + 1] > soff[j]]
                recorded = {}
                waits = []
                first_tier = {}
                for i, (kind, ax, ev, onx, arg, peer) in enumerate(ops):
                    if kind == OP_RECORD and ev == EV_XCH and ax == a and onx == 1:
                        recorded[arg] = i
                    if kind == OP_WAIT and ev == EV_XCH and ax == a and onx == 0:
                        waits.append((i, arg))
                    if kind == OP_TIER and arg not in first_tier:
                        first_tier[arg] = i
                for i, jp in waits:
                    assert jp in nonempty, "wait on an empty message %d" % jp
                    assert jp in recorded and recorded[jp] < i, "wait on message %d before its exchange" % jp
                # every non-empty message after the first must wait for its predecessor
                for prev, jj in zip(nonempty, nonempty[1:]):
                    t0 = lo[jj]
                    assert any(jp == prev and i < first_tier[t0] for i, jp in waits), \
                        "rank %d axis %d: message %d does not wait for %d" % (r, a, jj, prev)
                assert len(waits) == max(0, len(nonempty) - 1)


@pytest.mark.parametrize("world,owner", [(2, 0), (4, 0), (8, 0), (8, 1)])
def test_rank_digests_partition_the_table(oracle, world, owner):
    """bench.py at N > 1 names a wrong rank by comparing each rank's gm_digest (its own
    blocks) with the oracle's digest over the same blocks (oracle_dense_digest_blocks on
    the rank's GM_PLAN_OWN list).  The OWN lists partition the table, so those per-rank
    oracle digests sum to the full-table digest; and rank_digest_check accepts them."""
    import ctypes
    import os
    import sys
    heaps, root = 6, (1 << 24) - 1
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    rec = oracle.subtract_dense_mt(heaps)
    L = bench._oracle()
    seen = np.zeros(1 << (4 * (heaps - 3)), dtype=np.int64)
    per, total = [], 0
    for r in range(world):
        own = np.ascontiguousarray(_lib.dist_plan(heaps, world, r, _lib.PLAN_OWN, owner=owner)[1], dtype=np.uint32)
        seen[own] += 1
        d, c = ctypes.c_uint64(), ctypes.c_uint64()
        L.oracle_dense_digest_blocks(rec.ctypes.data, heaps, 3, ctypes.c_uint64(root), own.ctypes.data,
                                     ctypes.c_uint64(len(own)), 0, ctypes.byref(d), ctypes.byref(c))
        per.append((d.value, c.value))
        total = (total + d.value) & ((1 << 64) - 1)
    assert (seen == 1).all()
    assert (total, sum(c for _, c in per)) == (oracle.dense_digest(rec), 16 ** heaps)
    chk = bench.rank_digest_check(heaps, world, root, per, 4, 4, 1, owner)
    assert chk["wrong_ranks"] == [] and len(chk["ranks"]) == world
    bad = list(per)
    bad[world - 1] = (bad[world - 1][0] ^ 1, bad[world - 1][1])
    assert bench.rank_digest_check(heaps, world, root, bad, 4, 4, 1, owner)["wrong_ranks"] == [world - 1]


def _hang_rank(rank, world, phase, port):
    import os
    import time
    import torch.distributed as tdist
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    phase("exchange")
    if rank == 1:
        phase("stuck on purpose")
        while True:          # never reaches the collective: rank 0's all_reduce waits for ever
            time.sleep(1)
    import torch
    t = torch.ones(1)
    tdist.all_reduce(t)
    return float(t.item())


def test_rank_runner_stops_a_hung_rank():
    """The multi-process runner of the RCCL GPU tests (tests/mp_ranks.py): a gloo rank that
    hangs on purpose ends the run at its deadline, every rank process is gone, and the
    failure names each rank's last phase."""
    import time
    from mp_ranks import RankFailure, run_ranks
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    t = time.monotonic()
    with pytest.raises(RankFailure, match=r"timeout.*0=exchange, 1=stuck on purpose"):
        run_ranks(_hang_rank, 2, (port,), timeout=20, grace=3)
    assert time.monotonic() - t < 60


def _ok_rank(rank, world, phase, port):
    import os
    import torch
    import torch.distributed as tdist
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    t = torch.ones(1) * (rank + 1)
    tdist.all_reduce(t)
    return float(t.item())


def test_rank_runner_collects_results():
    from mp_ranks import run_ranks
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    assert run_ranks(_ok_rank, 3, (port,), timeout=60) == [6.0, 6.0, 6.0]
