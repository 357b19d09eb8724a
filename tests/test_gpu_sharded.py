"""GPU parity of the sharded (multi-GPU) algorithms on ONE device.

GM_OPT_VIRTUAL_RANKS runs G ranks inside one context: the same partition, block / box
lists, halo / all-to-all schedule and kernels as the one-process-per-GPU RCCL
path, with the exchanges done by device copies (dist_sub.hip, dist_sparse.hip) or by the tier
kernel's direct stores into the receiving rank's table (dist_box.hip).
Every sharded result must be bit-identical to the single-rank result.
"""
import ctypes

import numpy as np
import pytest

from conftest import digest, golden

from gamesmanmpi_amd import Context, _lib

pytestmark = pytest.mark.gpu

F2O, TTT, TOOT, OTH, SUB = 1, 2, 3, 4, 5


def _solve(game, params, ranks, root=None, engine=None, **opts):
    ctx = Context(game, params, device=0)
    if engine is not None:
        ctx.set_option(_lib.OPT_ENGINE, engine)
    for k, v in opts.items():
        ctx.set_option(getattr(_lib, "OPT_" + k.upper()), v)
    if ranks > 1:
        ctx.set_option(_lib.OPT_VIRTUAL_RANKS, ranks)
    if root is None:
        root = ctx.initial()
    n, rec = ctx.solve(root)
    return ctx, n, rec


@pytest.mark.parametrize("sym", [0, 1])
@pytest.mark.parametrize("heaps,ranks", [(4, 2), (5, 2), (5, 4), (6, 2), (6, 4), (6, 8), (7, 2), (7, 4), (7, 8)])
def test_dense_sharded_vs_oracle(oracle, heaps, ranks, sym):
    ref = oracle.subtract_dense(heaps)
    ctx, n, rec = _solve(SUB, (heaps,), ranks, dist_symmetry=sym)
    assert ctx.stats()["engine"] == _lib.ENGINE_DIST_DENSE
    k, r = ctx.export()
    assert n == 16 ** heaps
    assert np.array_equal(k, np.arange(16 ** heaps, dtype=np.uint64))
    assert np.array_equal(r, ref)


@pytest.mark.parametrize("batch,slots", [(1, 1), (1, 4), (2, 1), (3, 2), (4, 4), (8, 2), (16, 1), (100, 4)])
@pytest.mark.parametrize("ranks", [2, 8])
def test_dense_sharded_batches_and_rings(oracle, batch, slots, ranks):
    """Every halo batch size and send-ring depth gives the oracle's table (6 heaps: 46 tiers;
    at 2 ranks most halo blocks come from the symmetric fill, at 8 none)."""
    ref = oracle.subtract_dense(6)
    ctx, n, rec = _solve(SUB, (6,), ranks, dist_batch=batch, dist_slots=slots)
    k, r = ctx.export()
    assert np.array_equal(r, ref)


@pytest.mark.parametrize("heaps,ranks", [(5, 2), (6, 2), (6, 4), (7, 2), (7, 4), (7, 8)])
def test_dense_tier_balanced_vs_oracle(oracle, heaps, ranks):
    """GM_OPT_DIST_OWNER 1 (tier-balanced owner) gives the oracle's table."""
    ref = oracle.subtract_dense(heaps)
    ctx, n, rec = _solve(SUB, (heaps,), ranks, dist_owner=1)
    k, r = ctx.export()
    assert np.array_equal(k, np.arange(16 ** heaps, dtype=np.uint64))
    assert np.array_equal(r, ref)


@pytest.mark.parametrize("batch,slots", [(1, 1), (2, 4), (8, 2)])
def test_dense_tier_balanced_full_2_32_matches_single_gpu(batch, slots):
    single, n1, rec1 = _solve(SUB, (8,), 1)
    d1 = single.digest()
    single.close()
    for ranks in (2, 4, 8):
        ctx, n, rec = _solve(SUB, (8,), ranks, sub_interleave=10, dist_owner=1, dist_batch=batch,
                             dist_slots=slots)
        assert (n, rec) == (n1, rec1)
        assert ctx.digest() == d1
        # the halo blocks no heap permutation fills (tests/test_dist_plan.py pins the counts)
        assert ctx.stats()["exchanged_bytes"] == {2: 15, 4: 480, 8: 12896}[ranks] * 4096
        ctx.close()


def test_dense_sharded_custom_root(oracle):
    root = 0x3F0A5C
    ok, orec = oracle.solve(SUB, (6,), root=root)
    ctx, n, rec = _solve(SUB, (6,), 8, root=root)
    k, r = ctx.export()
    assert np.array_equal(k, ok) and np.array_equal(r, orec)
    assert ctx.query([root])[0] == rec


def test_dense_sharded_full_2_32_matches_single_gpu():
    """The block engine's sharded path (GM_OPT_SUB_INTERLEAVE 10) at full size."""
    single, n1, rec1 = _solve(SUB, (8,), 1)
    d1 = single.digest()
    single.close()
    halo = {2: 512 << 20, 4: 2 * (512 << 20), 8: 3 * (512 << 20)}   # full halo bytes per solve, all ranks
    for ranks in (2, 4, 8):
        for sym in (1, 0):
            ctx, n, rec = _solve(SUB, (8,), ranks, sub_interleave=10, dist_symmetry=sym)
            assert (n, rec) == (n1, rec1)
            assert ctx.digest() == d1
            sent = ctx.stats()["exchanged_bytes"]
            # the symmetric fill leaves 1/16, 1/8, 1/4 of the halo to cross the link
            want = halo[ranks] // {2: 16, 4: 8, 8: 4}[ranks] if sym else halo[ranks]
            assert sent == want, (ranks, sym, sent, want)
            ctx.close()


def _committed(name):
    import json
    import os
    from conftest import GOLDEN
    return json.load(open(os.path.join(GOLDEN, "oracle_digests.json")))[name]


def _plan_bytes(ranks, root=0xFFFFFFFF, **kw):
    """Halo bytes all ranks send per solve, from the plan (gm_box_plan GM_BOXPLAN_SEND)."""
    total = 0
    for r in range(ranks):
        for a in range(3):
            ent = _lib.box_plan(ranks, r, _lib.BOXPLAN_SEND, root=root, axis=a, **kw)
            total += int(sum(2048 if (int(e) >> 20) else 4096 for e in ent))
    return total


@pytest.mark.parametrize("sym", [1, 0])
@pytest.mark.parametrize("ranks", [2, 3, 4, 8])
def test_box_split_2_32_matches_oracle_digest(ranks, sym):
    """Config 5 on the box engine split over virtual ranks (csrc/dist_box.hip): every box on
    ONE rank, each rank on its own table (filled with 0xFF first, so a read of a box the rank
    neither computed nor received would show), halo boxes stored by the lower rank's tier kernel
    into the upper rank's table (an event per batch standing in for the signal; the solve
    replayed as one captured graph), crossing children read through heap transpositions of own boxes
    with the symmetric fill (sym 1) or all received (sym 0).  The ranks' digests sum to the C
    oracle's digest of the whole table, the root record is the oracle's, every rank computed
    its plan's boxes (summing to 2^20: work_vs_one_gpu = 1), and the bytes exchanged are the
    plan's."""
    ref = _committed("subtract_8")
    ctx, n, rec = _solve(SUB, (8,), ranks, timing=1, dist_symmetry=sym)
    st = ctx.stats()
    assert st["engine"] == _lib.ENGINE_DIST_DENSE and st["world"] == ranks
    assert (n, rec) == (1 << 32, ref["root_record"])
    assert ctx.digest() == (ref["digest"], 1 << 32)
    rs = ctx.rank_stats()
    want = [int(_lib.box_plan(ranks, r, _lib.BOXPLAN_COUNTS, symmetry=sym)[0]) for r in range(ranks)]
    assert [r["boxes"] for r in rs] == want and sum(want) == 1 << 20
    assert st["exchanged_bytes"] == _plan_bytes(ranks, symmetry=sym) > 0
    # every virtual rank's table together answers every key
    keys = np.array([0xFFFFFFFF, 0, 0x12345678, 0xFEDCBA98, 0x0F0F0F0F, 0x88888888], dtype=np.uint64)
    single, _, _ = _solve(SUB, (8,), 1)
    assert np.array_equal(ctx.query(keys), single.query(keys))
    single.close()
    ctx.close()


@pytest.mark.parametrize("ranks", [2, 8])
def test_box_split_graph_and_eager_launches(ranks, monkeypatch):
    """The split solve's launches captured once and replayed as a graph (GM_OPT_GRAPH 1, the
    default), launched eagerly (0), and replayed with the IPC transport's flag kernels in the
    lists (GM_BOX_SIGNAL_KERNELS=1, read when the plan is prepared): three solves each, every one
    the oracle's digest and the plan's halo bytes; a solo rank's replay (its own graph) too."""
    ref = _committed("subtract_8")
    want = _plan_bytes(ranks)
    for graph, sigk in ((1, None), (0, None), (1, "1")):
        if sigk:
            monkeypatch.setenv("GM_BOX_SIGNAL_KERNELS", sigk)
        else:
            monkeypatch.delenv("GM_BOX_SIGNAL_KERNELS", raising=False)
        ctx = Context(SUB, (8,), device=0)
        ctx.set_option(_lib.OPT_GRAPH, graph)
        ctx.set_option(_lib.OPT_VIRTUAL_RANKS, ranks)
        for _ in range(3):
            n, rec = ctx.solve(0xFFFFFFFF)
            assert (n, rec) == (1 << 32, ref["root_record"])
            assert ctx.digest() == (ref["digest"], 1 << 32), (graph, sigk)
            assert ctx.stats()["exchanged_bytes"] == want
        ctx.set_option(_lib.OPT_DIST_SOLO, ranks)   # the top rank alone: the others' boxes stand in
        ctx.set_option(_lib.OPT_TIMING, 1)
        for _ in range(2):
            ctx.solve(0xFFFFFFFF)
            assert ctx.rank_stats()[ranks - 1]["kernel_ms"] > 0
        ctx.set_option(_lib.OPT_DIST_SOLO, 0)
        ctx.solve(0xFFFFFFFF)
        assert ctx.digest() == (ref["digest"], 1 << 32)
        ctx.close()


def test_box_four_wave_thin_tiers(monkeypatch):
    """GM_BOX_THIN_GROUPS (development): box-tiers of at most that many groups run the four-wave
    kernel (box_tier4_kernel) -- at N = 1 and on every split variant (messages, direct stores,
    with and without fills) -- and every table is still the oracle's."""
    ref = _committed("subtract_8")
    monkeypatch.setenv("GM_BOX_THIN_GROUPS", "1000")
    for ranks, sym in ((1, 1), (2, 1), (8, 1), (8, 0)):
        ctx, n, rec = _solve(SUB, (8,), ranks, dist_symmetry=sym)
        assert (n, rec) == (1 << 32, ref["root_record"])
        assert ctx.digest() == (ref["digest"], 1 << 32), (ranks, sym)
        ctx.close()


def test_box_split_comparisons_2_32_matches_oracle_digest():
    """GM_OPT_BOX_SPLIT 1 (tier-balanced comparisons; not the default, tests/test_box_plan.py
    says why) gives the oracle's digest at 2, 4 and 8 ranks."""
    ref = _committed("subtract_8")
    for ranks in (2, 4, 8):
        ctx, n, rec = _solve(SUB, (8,), ranks, box_split=1)
        assert (n, rec) == (1 << 32, ref["root_record"])
        assert ctx.digest() == (ref["digest"], 1 << 32)
        ctx.close()


_ORACLE_ROOTS = {}


def _oracle_root(oracle, root):
    if root not in _ORACLE_ROOTS:
        _ORACLE_ROOTS[root] = oracle.solve(SUB, (8,), root=root)
    return _ORACLE_ROOTS[root]


@pytest.mark.parametrize("batch", [1, 2, 3, 8, 100])
def test_box_split_batches(oracle, batch):
    """Every halo batch size gives the oracle's table (8 ranks, root 0x33557777: 2.4 M positions)."""
    root = 0x33557777
    ok, orec = _oracle_root(oracle, root)
    ctx, n, rec = _solve(SUB, (8,), 8, root=root, dist_batch=batch)
    k, r = ctx.export()
    assert np.array_equal(k, ok) and np.array_equal(r, orec)
    ctx.close()


@pytest.mark.parametrize("ranks", [2, 4, 8])
@pytest.mark.parametrize("root", [0x33337777, 0x33557777, 0x333337BF, 0x13572468])
def test_box_split_custom_roots_vs_oracle(oracle, ranks, root):
    """Custom roots on the split box engine (axes chosen among the heaps the region splits;
    0x13572468 leaves ranks without boxes at 8).  Export, digest and query equal the C
    oracle's table; keys outside the root's region query as unsolved."""
    ok, orec = _oracle_root(oracle, root)
    ctx, n, rec = _solve(SUB, (8,), ranks, root=root)
    assert n == len(ok)
    k, r = ctx.export()
    assert np.array_equal(k, ok) and np.array_equal(r, orec)
    assert ctx.digest() == (digest(ok, orec), len(ok))
    sample = ok[:: max(1, len(ok) // 5000)]
    assert np.array_equal(ctx.query(sample), orec[:: max(1, len(ok) // 5000)])
    outside = np.array([root + 1 if (root & 15) < 15 else root | 0xF0000000, 0x1FFFFFFFF], dtype=np.uint64)
    assert ctx.query(outside).tolist() == [_lib.REC_UNSOLVED] * 2
    ctx.close()


def test_box_split_solo_timing():
    """GM_OPT_DIST_SOLO r + 1 (loopback): rank r's op list alone, its cross-rank waits dropped,
    the other ranks' messages of the previous full solve standing in, queued whole behind a
    hold of the stream -- its own GPU critical path, per op (gm_rank_op_ms) and from its first
    tier launch to its last (gm_rank_stats)."""
    ctx, n, rec = _solve(SUB, (8,), 8, timing=2)
    for r in (0, 7):
        ctx.set_option(_lib.OPT_DIST_SOLO, r + 1)
        ctx.set_option(_lib.OPT_TIMING, 1)      # the span alone
        ctx.solve(0xFFFFFFFF)
        span1 = ctx.rank_stats()[r]["kernel_ms"]
        assert span1 > 0 and (ctx.rank_op_ms(r) == 0).all()
        ctx.set_option(_lib.OPT_TIMING, 2)      # and per op
        ctx.solve(0xFFFFFFFF)
        ms = ctx.rank_op_ms(r)
        ops = _lib.box_plan(8, r, _lib.BOXPLAN_OPS, loopback=1).reshape(-1, 6)
        assert len(ms) == len(ops)
        kind = ops[:, 0]
        tier = kind == _lib.BOP_TIER
        assert (ms[tier] > 0).all()
        assert (ms[(kind == _lib.BOP_RECORD) | (kind == _lib.BOP_WAIT)] == 0).all()
        span = ctx.rank_stats()[r]["kernel_ms"]
        # the list was queued whole behind the hold; the per-op event pairs only add time
        assert ms[tier].sum() <= span + 1e-3 and span1 <= 1.1 * span + 0.01
    ctx.set_option(_lib.OPT_DIST_SOLO, 0)
    ref = _committed("subtract_8")
    n, rec = ctx.solve(0xFFFFFFFF)
    assert ctx.digest() == (ref["digest"], 1 << 32)
    ctx.close()


@pytest.mark.parametrize("root", [0xFFFFFFFF, 0x33337777, 0x000F0FFF, 0x9ABCDEF1])
def test_box_dataflow_on_one_gpu_vs_oracle(oracle, root):
    """GM_OPT_BOX_FLOW 1 on one GPU: the whole box-tier chain in one launch, each box group
    waiting for its child boxes' flags (csrc/dense_box.hip box_flow_kernel), equals the
    tier launches and, for the full table, the committed C-oracle digest; twice in a row
    (the second solve's epoch must not accept the first solve's flags)."""
    tiers, n0, r0 = _solve(SUB, (8,), 1, root=root, box_flow=0)
    d0 = tiers.digest()
    tiers.close()
    ctx, n, rec = _solve(SUB, (8,), 1, root=root, box_flow=1, timing=1)
    assert ctx.stats()["kernel_launches"] == 1 and ctx.stats()["flow_fallbacks"] == 0
    assert (n, rec, ctx.digest()) == (n0, r0, d0)
    n2, rec2 = ctx.solve(root)
    assert (n2, rec2, ctx.digest()) == (n0, r0, d0)
    if root == 0xFFFFFFFF:
        ref = _committed("subtract_8")
        assert d0 == (ref["digest"], 1 << 32) and r0 == ref["root_record"]
    elif root < 16 ** 7:
        k, r = ctx.export()
        assert np.array_equal(r, oracle.subtract_dense_mt(7)[k.astype(np.int64)])
    ctx.close()


_FLOW_RUN = """
import json, os, sys
sys.path.insert(0, sys.argv[1])
from gamesmanmpi_amd import Context, _lib
ref = json.load(open(os.path.join(sys.argv[1], "tests", "golden", "oracle_digests.json")))["subtract_8"]
ctx = Context(5, (8,), device=0)
ctx.set_option(_lib.OPT_BOX_FLOW, 1)
ctx.set_option(_lib.OPT_TIMING, 1)
out = []
for rep in range(2):
    n, rec = ctx.solve(0xFFFFFFFF)
    assert ctx.digest() == (ref["digest"], 1 << 32) and rec == ref["root_record"], rep
    st = ctx.stats()
    out.append((st["kernel_launches"], st["flow_fallbacks"]))
print(json.dumps(out))
"""


def _flow_run(**env):
    import json
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _FLOW_RUN, repo], env=dict(os.environ, **env), capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1]), r.stderr


def test_box_dataflow_timeout_falls_back_to_tier_launches():
    """A dataflow wait that outlasts its limit (GM_BOX_FLOW_TEST_STALL makes every wait look
    for an epoch no flag holds; GM_BOX_FLOW_TIMEOUT_MS 20) ends the launch -- every wave sees
    the error and leaves -- and the solve is redone with tier launches: the oracle's digest, a
    line on stderr, gm_stats_t.flow_fallbacks 1, and tier launches from then on (fresh process:
    the hooks are read at launch capture)."""
    out, err = _flow_run(GM_BOX_FLOW_TEST_STALL="1", GM_BOX_FLOW_TIMEOUT_MS="20")
    assert out == [[41, 1], [41, 1]]
    assert "re-solving with tier launches" in err


def test_box_dataflow_grid_from_occupancy():
    """the dataflow launch's grid is the kernel's resident capacity from
    the occupancy API, not a constant.  With 48 KiB of extra dynamic LDS per workgroup
    (GM_BOX_FLOW_EXTRA_LDS) fewer workgroups fit a CU; the launch shrinks to what is resident,
    so every wait makes progress: one launch, no fallback, the oracle's digest."""
    out, err = _flow_run(GM_BOX_FLOW_EXTRA_LDS=str(48 << 10))
    assert out == [[1, 0], [1, 0]], err
    assert "re-solving" not in err


def test_box_engine_query_outside_the_root_region_is_unsolved():
    """the box engine solves only the boxes of the root's region and never clears
    the table, so a key with a nibble above the root's must query as 0xFFFF, not as whatever
    the slot holds (include/gmsolve.h gm_query)."""
    ctx, _, _ = _solve(SUB, (8,), 1)   # writes every slot; the next solve reuses the memory
    root = 0x3F0A5C12
    ctx.solve(root)
    inside = np.array([root, 0x3F0A5C02, 0], dtype=np.uint64)
    outside = np.array([0x3F0A5C13, 0x4F0A5C12, 0xFFFFFFFF, 1 << 32], dtype=np.uint64)
    assert (ctx.query(inside) != _lib.REC_UNSOLVED).all()
    assert ctx.query(outside).tolist() == [_lib.REC_UNSOLVED] * 4
    ctx.close()


@pytest.mark.parametrize("ranks", [2, 3, 8])
@pytest.mark.parametrize("name,game,params,root", [
    ("ttt", TTT, (), None), ("othello_4x4", OTH, (4, 4), None), ("toot_4x3", TOOT, (4, 3), None),
    ("four_to_one_six", F2O, (), 6)])
def test_sparse_sharded_vs_golden(name, game, params, root, ranks):
    keys, recs = golden(name)
    ctx, n, rec = _solve(game, params, ranks, root=root, engine=_lib.ENGINE_SPARSE)
    k, r = ctx.export()
    assert n == len(keys)
    assert np.array_equal(k, keys) and np.array_equal(r, recs)
    assert ctx.digest() == (digest(keys, recs), len(keys))


def test_sparse_sharded_toot_4x4_vs_oracle(oracle):
    ok, orec = oracle.solve(TOOT, (4, 4))
    ctx, n, rec = _solve(TOOT, (4, 4), 8)
    assert ctx.digest() == (digest(ok, orec), len(ok))


@pytest.mark.slow
def test_sparse_sharded_toot_6x4_matches_single_gpu():
    single, n1, rec1 = _solve(TOOT, (6, 4), 1)
    d1 = single.digest()
    counts1 = single.tier_counts().tolist()
    single.close()
    ctx, n, rec = _solve(TOOT, (6, 4), 8)
    assert (n, rec) == (n1, rec1) and n == 1187212827
    assert ctx.tier_counts().tolist() == counts1
    assert ctx.digest() == d1


def _rccl_one_rank(game, params):
    ctx = Context(game, params, device=0)
    buf = ctypes.create_string_buffer(128)
    _lib.check(_lib.lib().gm_comm_unique_id(buf, 128))
    ctx.set_comm(0, 1, buf.raw)
    ctx.set_option(_lib.OPT_ENGINE, _lib.ENGINE_DIST_SPARSE)
    n, rec = ctx.solve(ctx.initial())
    assert ctx.stats()["engine"] == _lib.ENGINE_DIST_SPARSE
    return ctx, n, rec


@pytest.mark.parametrize("name,game,params", [("othello_4x4", OTH, (4, 4)), ("toot_4x3", TOOT, (4, 3)),
                                              ("ttt", TTT, ())])
def test_sparse_rccl_transport_one_rank(name, game, params):
    """The hash-sharded engine's RCCL transport on one GPU: over a one-rank communicator
    every exchange is a real ncclGroup of self send/recv, the counts an ncclAllGather and
    the tier totals an ncclAllReduce; the table equals the reference plugin's golden one."""
    ctx, n, rec = _rccl_one_rank(game, params)
    keys, recs = golden(name)
    k, r = ctx.export()
    assert n == len(keys)
    assert np.array_equal(k, keys) and np.array_equal(r, recs)
    ctx.close()


def test_sparse_rccl_transport_one_rank_toot_6x4():
    """Config 3 at full size through the RCCL transport (one rank): per-ply counts and the
    full-table digest equal the one-GPU engine's."""
    single, n1, rec1 = _solve(TOOT, (6, 4), 1)
    d1, c1 = single.digest(), single.tier_counts().tolist()
    single.close()
    ctx, n, rec = _rccl_one_rank(TOOT, (6, 4))
    assert (n, rec) == (n1, rec1) and n == 1187212827
    assert ctx.tier_counts().tolist() == c1
    assert ctx.digest() == d1
    ctx.close()


@pytest.mark.parametrize("ranks", [2, 4, 8])
def test_box_split_dataflow_2_32_matches_oracle_digest(ranks):
    """GM_OPT_BOX_FLOW 1 on the split box engine (csrc/dense_box.hip box_split_flow_kernel):
    every virtual rank's whole chain in ONE launch with the others' (workgroup w runs rank
    w % G), the halo boxes stored straight into the receiving rank's table and their flags
    into its flag array, a box starting when its child boxes' flags -- own or received -- hold
    the solve's epoch.  Twice in a row (epochs): the committed 2^32 oracle digest, the root
    record, one launch per solve, the plan's halo bytes."""
    ref = _committed("subtract_8")
    ctx, n, rec = _solve(SUB, (8,), ranks, timing=1, box_flow=1)
    for _ in range(2):
        assert (n, rec) == (1 << 32, ref["root_record"])
        assert ctx.digest() == (ref["digest"], 1 << 32)
        st = ctx.stats()
        assert st["kernel_launches"] == 1 and st["exchanged_bytes"] == _plan_bytes(ranks) > 0
        n, rec = ctx.solve(0xFFFFFFFF)
    ctx.close()


@pytest.mark.parametrize("root", [0x33557777, 0x13572468])
def test_box_split_dataflow_custom_roots_vs_oracle(oracle, root):
    """The split dataflow at 8 virtual ranks on custom roots (0x13572468 leaves ranks idle):
    export equals the C oracle's table."""
    ok, orec = _oracle_root(oracle, root)
    ctx, n, rec = _solve(SUB, (8,), 8, root=root, box_flow=1)
    k, r = ctx.export()
    assert np.array_equal(k, ok) and np.array_equal(r, orec)
    ctx.close()


def test_box_split_dataflow_solo_rank():
    """GM_OPT_DIST_SOLO with the split dataflow: one rank's launch alone, the boxes it
    receives marked stored for the solve's epoch (the previous full solve wrote them) -- its
    own dataflow critical path; the full solve after it still equals the oracle."""
    ref = _committed("subtract_8")
    ctx, n, rec = _solve(SUB, (8,), 8, timing=1, box_flow=1)
    for r in (0, 7):
        ctx.set_option(_lib.OPT_DIST_SOLO, r + 1)
        ctx.solve(0xFFFFFFFF)
        assert ctx.rank_stats()[r]["kernel_ms"] > 0
    ctx.set_option(_lib.OPT_DIST_SOLO, 0)
    ctx.solve(0xFFFFFFFF)
    assert ctx.digest() == (ref["digest"], 1 << 32)
    ctx.close()
