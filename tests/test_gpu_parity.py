"""GPU parity: libgmsolve.so on the MI355X against the golden tables and the C oracle.

Every comparison is bit-exact on (key, value, remoteness).  Fixtures come from
the reference's own plugins (tests/golden/make_golden.py); larger cases compare
with the C oracle (oracle/gm_oracle.c), which is itself pinned to the fixtures
by tests/test_oracle_golden.py; full-size cases use size-independent properties
(closed-form values, the reference-independent per-ply counts of SURVEY App. D).
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, digest, golden, load_plugin

pytestmark = pytest.mark.gpu

from gamesmanmpi_amd import Context, Solver, _lib, games  # noqa: E402

F2O, TTT, TOOT, OTH, SUB = 1, 2, 3, 4, 5


def _solve(game, params=(), root=None, engine=None, **opts):
    ctx = Context(game, params, device=0)
    if engine is not None:
        ctx.set_option(_lib.OPT_ENGINE, engine)
    for k, v in opts.items():
        ctx.set_option(getattr(_lib, "OPT_" + k.upper()), v)
    if root is None:
        root = ctx.initial()
    n, rec = ctx.solve(root)
    return ctx, n, rec


def test_device_visible():
    assert _lib.lib().gm_device_count() >= 1


@pytest.mark.parametrize("engine", [_lib.ENGINE_DENSE, _lib.ENGINE_SPARSE])
def test_ttt_full_table(engine):
    keys, recs = golden("ttt")
    ctx, n, rec = _solve(TTT, engine=engine)
    k, r = ctx.export()
    assert n == len(keys) == 5478
    assert np.array_equal(k, keys) and np.array_equal(r, recs)
    assert rec == (2 << 14) | 9          # TIE in 9
    assert ctx.digest() == (digest(keys, recs), len(keys))


@pytest.mark.parametrize("case", ["four", "six", "one", "zero"])
def test_four_to_one_roots(case):
    keys, recs = golden("four_to_one_" + case)
    root = {"four": 4, "six": 6, "one": 1, "zero": 0}[case]
    ctx, n, rec = _solve(F2O, root=root)
    k, r = ctx.export()
    assert np.array_equal(k, keys) and np.array_equal(r, recs)


def test_othello_4x4():
    keys, recs = golden("othello_4x4")
    ctx, n, rec = _solve(OTH, (4, 4))
    k, r = ctx.export()
    assert n == 54089
    assert np.array_equal(k, keys) and np.array_equal(r, recs)
    assert rec == (1 << 14) | 12         # LOSS in 12


@pytest.mark.parametrize("ranks", [1, 4])
def test_othello_custom_roots_vs_oracle(oracle, ranks):
    """Othello 4x4 from positions two and four plies in (the launcher's --custom path),
    one GPU and hash-sharded, against the C oracle."""
    hd = games.HostDescriptor(games.OthelloCodec(4, 4))
    level = [hd.initial()]
    for ply in range(1, 5):
        level = sorted({c for k in level for c in hd.expand(k)[1]})
        if ply in (2, 4):
            r = level[len(level) // 2]
            ok, orec = oracle.solve(OTH, (4, 4), root=r)
            ctx = Context(OTH, (4, 4), device=0)
            if ranks > 1:
                ctx.set_option(_lib.OPT_VIRTUAL_RANKS, ranks)
            n, rec = ctx.solve(r)
            k, rr = ctx.export()
            assert n == len(ok) and np.array_equal(k, ok) and np.array_equal(rr, orec)
            ctx.close()
    hd.close()


@pytest.mark.parametrize("game,params,name", [(OTH, (4, 4), "othello_4x4"), (TOOT, (4, 3), "toot_4x3"),
                                              (F2O, (), "four_to_one_six")])
def test_sparse_replay_is_identical(game, params, name):
    """A repeated solve of the same (game, parameters, root) replays the recorded tier
    sequence as one graph with no host round trip (csrc/sparse.hip replay_with); every
    replay must give the golden table, and a different root must not reuse the record."""
    keys, recs = golden(name)
    ctx = Context(game, params, device=0)
    root = 6 if game == F2O else ctx.initial()
    first = None
    for i in range(4):
        n, rec = ctx.solve(root)
        k, r = ctx.export()
        assert n == len(keys) and np.array_equal(k, keys) and np.array_equal(r, recs), i
        assert ctx.digest() == (digest(keys, recs), len(keys))
        st = ctx.stats()   # a replay reports the recorded solve's counts, not zeros
        counts = (st["n_positions"], st["n_tiers"], st["n_edges"], st["algo_bytes"], st["table_bytes"])
        first = first or counts
        assert counts == first and st["n_edges"] > 0, i
    if game == F2O:   # another root: a fresh synced solve, then its own replays
        k4, r4 = golden("four_to_one_four")
        for i in range(2):
            ctx.solve(4)
            k, r = ctx.export()
            assert np.array_equal(k, k4) and np.array_equal(r, r4), i
        ctx.solve(6)
        k, r = ctx.export()
        assert np.array_equal(k, keys) and np.array_equal(r, recs)


def test_sparse_replay_after_another_engine_restores_counts():
    """A replay restores the recorded solve's position count and per-tier counts, also
    when another engine solved a different root on the same context in between
    (csrc/sparse.hip replay_with): sparse A, dense B, sparse A again."""
    keys, recs = golden("ttt")
    ctx = Context(TTT, (), device=0)
    a = ctx.initial()
    ctx.set_option(_lib.OPT_ENGINE, _lib.ENGINE_SPARSE)
    n1, r1 = ctx.solve(a)
    t1 = ctx.tier_counts().tolist()
    assert n1 == len(keys) == sum(t1)
    b = 1 + 3 * 2 + 9 * 1   # X at 0, O at 1, X at 2: a custom root deeper in the game
    ctx.set_option(_lib.OPT_ENGINE, _lib.ENGINE_DENSE)
    nb, _ = ctx.solve(b)
    assert nb < n1
    ctx.set_option(_lib.OPT_ENGINE, _lib.ENGINE_SPARSE)
    for _ in range(2):   # the second solve of A is a replay
        n2, r2 = ctx.solve(a)
        assert (n2, r2) == (n1, r1) and ctx.tier_counts().tolist() == t1
        assert ctx.stats()["n_positions"] == n1
        k, r = ctx.export()
        assert np.array_equal(k, keys) and np.array_equal(r, recs)


def test_sparse_replay_is_faster():
    """Othello 4x4 (54,089 positions): the replay has no per-tier host round trip."""
    ctx = Context(OTH, (4, 4), device=0)
    root = ctx.initial()
    ctx.solve(root)
    first = ctx.stats()["solve_ms"]
    best = min((ctx.solve(root), ctx.stats()["solve_ms"])[1] for _ in range(5))
    assert best < first


@pytest.mark.parametrize("dims", [(3, 3), (4, 3)])
def test_toot_small_boards(dims):
    keys, recs = golden("toot_%dx%d" % dims)
    ctx, n, rec = _solve(TOOT, dims)
    k, r = ctx.export()
    assert np.array_equal(k, keys) and np.array_equal(r, recs)


def test_toot_4x4_vs_oracle(oracle):
    ok, orec = oracle.solve(TOOT, (4, 4))
    assert len(ok) == 3468773
    ctx, n, rec = _solve(TOOT, (4, 4))
    assert n == len(ok)
    assert ctx.digest() == (digest(ok, orec), len(ok))
    k, r = ctx.export()
    assert np.array_equal(k, ok) and np.array_equal(r, orec)


@pytest.mark.parametrize("heaps", [1, 2, 3, 4, 5])
@pytest.mark.parametrize("low", [1, 2, 3])
def test_subtract_dense_vs_oracle(oracle, heaps, low):
    ref = oracle.subtract_dense(heaps)
    ctx, n, rec = _solve(SUB, (heaps,), sub_low=low)
    k, r = ctx.export()
    assert n == 16 ** heaps
    assert np.array_equal(k, np.arange(16 ** heaps, dtype=np.uint64))
    assert np.array_equal(r, ref)


@pytest.mark.parametrize("variant", [1, 6, 10])
@pytest.mark.parametrize("heaps", [3, 4, 5, 6])
def test_subtract_kernel_variants_vs_oracle(oracle, heaps, variant):
    """Dense kernel options (GM_OPT_SUB_INTERLEAVE 1 = one block per workgroup, 6 = four-block
    kernel, 10 = walker (default below 8 heaps)) against the oracle."""
    ref = oracle.subtract_dense(heaps)
    ctx, n, rec = _solve(SUB, (heaps,), sub_interleave=variant)
    assert np.array_equal(ctx.export()[1], ref)


@pytest.mark.parametrize("order", [0, 1, 2])
@pytest.mark.parametrize("heaps", [5, 6])
def test_subtract_block_orders_vs_oracle(oracle, heaps, order):
    """Block order inside a tier (GM_OPT_SUB_ORDER 0 key, 1 Morton, 2 Hilbert,
    csrc/dense_sub.hip sort_tiers_morton) changes only which
    workgroup solves which block: the table must not change."""
    ref = oracle.subtract_dense(heaps)
    ctx, n, rec = _solve(SUB, (heaps,), sub_order=order)
    assert np.array_equal(ctx.export()[1], ref)


@pytest.mark.parametrize("variant", [10, 20])
def test_subtract_kernel_variants_full_2_32_match(variant):
    a, n1, r1 = _solve(SUB, (8,), sub_interleave=6)
    d1 = a.digest()
    a.close()
    b, n2, r2 = _solve(SUB, (8,), sub_interleave=variant)
    assert (n2, r2) == (n1, r1) and b.digest() == d1


_WALKER_EVERYWHERE = r'''
import ctypes, os, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from gamesmanmpi_amd import Context, _lib
ol = ctypes.CDLL(os.path.join(sys.argv[1], "oracle", "_build", "liboracle.so"))
ol.oracle_subtract_dense.argtypes = [ctypes.c_int, ctypes.c_void_p]
for heaps, variant in [(h, 10) for h in (3, 4, 5, 6)]:
    ctx = Context(_lib.GAME_SUBTRACT, (heaps,), device=0)
    ctx.set_option(_lib.OPT_SUB_INTERLEAVE, variant)
    ctx.solve(ctx.initial())
    ref = np.empty(16 ** heaps, dtype=np.uint16)
    assert ol.oracle_subtract_dense(heaps, ref.ctypes.data) == 0
    assert np.array_equal(ctx.export()[1], ref), heaps
    ctx.close()
print("ok")
'''


def test_walker_kernel_on_every_tier_vs_oracle():
    """The walker kernel runs only tiers of >= GM_WK_MIN blocks (smaller ones take the b4
    kernel); with GM_WK_MIN=0 it solves every tier of the 3..6-heap games (fresh process:
    the threshold is read once)."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GM_WK_MIN="0")
    r = subprocess.run([sys.executable, "-c", _WALKER_EVERYWHERE, repo], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr


_SPARSE_BATCH_EVERYWHERE = r'''
import json, os, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
sys.path.insert(0, os.path.join(sys.argv[1], "tests"))
from conftest import golden, digest
from gamesmanmpi_amd import Context, _lib
for name, game, params in [("othello_4x4", 4, (4, 4)), ("toot_4x3", 3, (4, 3)), ("ttt", 2, ())]:
    keys, recs = golden(name)
    for sym in (1, 0):
        ctx = Context(game, params, device=0)
        ctx.set_option(_lib.OPT_ENGINE, _lib.ENGINE_SPARSE)
        ctx.set_option(_lib.OPT_SYMMETRY, sym)
        for rep in range(2):   # the synced solve, then the replay (its sorts run in the graph)
            n, rec = ctx.solve(ctx.initial())
            k, r = ctx.export()
            assert n == len(keys) and np.array_equal(k, keys) and np.array_equal(r, recs), (name, sym, rep)
        ctx.close()
ref = json.load(open(os.path.join(sys.argv[1], "tests", "golden", "oracle_digests.json")))["toot_4x4"]
ctx = Context(3, (4, 4), device=0)
for rep in range(2):
    n, rec = ctx.solve(ctx.initial())
    assert ctx.digest() == (ref["digest"], ref["positions"]) and rec == ref["root_record"], rep
print("ok")
'''


@pytest.mark.parametrize("split_max,mode", [("1", "1"), ("4096", "1"), ("4096", "3"), ("1", "0")])
def test_sparse_sorted_lists_everywhere_vs_golden(split_max, mode):
    """The sparse engine's sorted interior lists (radix-sorted by the key's top bits, then
    the plain expand / retro kernels: GM_SPARSE_BATCH 1, the default; 3: 1 with every
    sorted pair checked on the device; 0: unsorted; csrc/sparse.hip) apply only to
    tiers of >= 65,536 interior positions; GM_SPARSE_SPLIT_MAX moves them onto every tier
    (1) or the mid-size ones of these games (4096), synced solve and replay, with and
    without the symmetry reduction: the reference plugins' golden tables and the Toot 4x4
    oracle digest (fresh process: the knobs are read once)."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GM_SPARSE_SPLIT_MAX=split_max, GM_SPARSE_BATCH=mode)
    r = subprocess.run([sys.executable, "-c", _SPARSE_BATCH_EVERYWHERE, repo], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr


@pytest.mark.parametrize("split_max", ["1", "4096"])
def test_sparse_csr_retro_vs_golden(split_max):
    """GM_SPARSE_CSR=1 (csrc/sparse.hip expand_csr_kernel / retro_csr_kernel: expand records its
    undecided children's table slots, retro reads them instead of regenerating and probing)
    on every tier of these games that takes the plain kernels: the reference plugins' golden
    tables and the Toot 4x4 oracle digest, synced solve and replay (fresh process)."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GM_SPARSE_CSR="1", GM_SPARSE_SPLIT_MAX=split_max)
    r = subprocess.run([sys.executable, "-c", _SPARSE_BATCH_EVERYWHERE, repo], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr


@pytest.mark.parametrize("home_w", ["16", "20"])
def test_sparse_locality_home_vs_golden(home_w):
    """GM_SPARSE_HOME_W (development knob, DESIGN.md §4.2: measured and not kept): the tier
    tables' locality home -- a key's group picks a base, a hash of the key one of 2^w slots
    from it -- gives the same tables: the golden tables and the Toot 4x4 oracle digest,
    synced solve and replay (fresh process: the knob is read once)."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GM_SPARSE_HOME_W=home_w, GM_SPARSE_SPLIT_MAX="4096")
    r = subprocess.run([sys.executable, "-c", _SPARSE_BATCH_EVERYWHERE, repo], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr


def test_subtract_graph_replay_is_identical(oracle):
    ref = oracle.subtract_dense(5)
    for graph in (0, 1, 1):
        ctx, n, rec = _solve(SUB, (5,), graph=graph)
        assert np.array_equal(ctx.export()[1], ref)


@pytest.mark.parametrize("heaps", [2, 3])
def test_subtract_sparse_engine_matches_generic_oracle(oracle, heaps):
    ok, orec = oracle.solve(SUB, (heaps,))
    ctx, n, rec = _solve(SUB, (heaps,), engine=_lib.ENGINE_SPARSE)
    k, r = ctx.export()
    assert np.array_equal(k, ok) and np.array_equal(r, orec)


def test_subtract_custom_root_box(oracle):
    # root 0x0A35: reachable set is the box h_i <= root_i
    root = 0x0A35
    ok, orec = oracle.solve(SUB, (4,), root=root)
    ctx, n, rec = _solve(SUB, (4,), root=root)
    k, r = ctx.export()
    assert n == len(ok) == 11 * 4 * 6 * 1
    assert np.array_equal(k, ok) and np.array_equal(r, orec)


@pytest.mark.parametrize("root", [0x00000003, 0x000F0FFF, 0x12345678])
def test_subtract_8_heaps_custom_root_solves_its_box_only(oracle, root):
    """The block engine (GM_OPT_SUB_INTERLEAVE 10) launches only the blocks inside the
    root's box (every high nibble <= the root's): a root with empty high heaps is one
    block, one launch.  Values are position-intrinsic, so the box equals the full 7-heap
    oracle table's entries where the top nibble is 0 (roots below 16^7)."""
    ctx, n, rec = _solve(SUB, (8,), root=root, timing=1, sub_interleave=10)
    box = 1
    for j in range(8):
        box *= ((root >> (4 * j)) & 15) + 1
    assert n == box
    blocks = 1
    for j in range(3, 8):
        blocks *= ((root >> (4 * j)) & 15) + 1
    st = ctx.stats()
    tiers = sum((root >> (4 * j)) & 15 for j in range(3, 8)) + 1
    assert st["kernel_launches"] == tiers, (st["kernel_launches"], tiers, blocks)
    if root < 16 ** 7:
        ref = oracle.subtract_dense_mt(7)
        k, r = ctx.export()
        assert len(k) == box and np.array_equal(r, ref[k.astype(np.int64)])
    else:
        g = 0
        for j in range(8):
            g ^= ((root >> (4 * j)) & 15) % 3
        assert (rec >> 14) == (1 if g == 0 else 0)


def _box_tiers(root):
    """Box-tiers of the box engine for a root: heaps 0-3 in quarters, 4-7 in halves."""
    return sum(((root >> (4 * j)) & 15) >> (2 if j < 4 else 1) for j in range(8)) + 1


@pytest.mark.parametrize("root", [0x00000003, 0x000F0FFF, 0x12345678, 0xFFFF0000, 0x0000FFFF, 0x9ABCDEF1, 0x7F7F7F7F, 0x0FFFFFFF])
def test_subtract_8_heaps_box_engine_custom_roots(oracle, root):
    """The box engine (GM_OPT_SUB_INTERLEAVE 20, the 8-heap default, csrc/dense_box.hip)
    launches one box-tier per sum of the root box's coordinates and equals the block
    engine on every root: same count, root record and digest; for roots below 16^7 the
    exported records equal the 7-heap C-oracle table (0x0FFFFFFF: 2^28 positions, the
    export's table-copy path; smaller boxes go through the device query)."""
    a, n1, r1 = _solve(SUB, (8,), root=root, timing=1, sub_interleave=20)
    assert a.stats()["kernel_launches"] == _box_tiers(root)
    da = a.digest()
    b, n2, r2 = _solve(SUB, (8,), root=root, sub_interleave=10)
    assert (n1, r1, da) == (n2, r2, b.digest())
    if root < 16 ** 7:
        ref = oracle.subtract_dense_mt(7)
        k, r = a.export()
        assert np.array_equal(r, ref[k.astype(np.int64)])


def test_subtract_single_heap_is_four_to_one():
    # one heap == Four-To-One for piles >= 0; golden from the reference plugin
    keys, recs = golden("four_to_one_six")
    ctx, n, rec = _solve(SUB, (1,), root=6)
    sub = dict(zip(*[a.tolist() for a in ctx.export()]))
    for k, r in zip(keys.tolist(), recs.tolist()):
        x = k - (1 << 64) if k >> 63 else k
        if x >= 0:
            assert sub[x] == r


def _closed_form_values(keys, heaps):
    g = np.zeros(len(keys), dtype=np.int64)
    for i in range(heaps):
        g ^= ((keys >> np.uint64(4 * i)) & np.uint64(15)).astype(np.int64) % 3
    return np.where(g == 0, 1, 0)   # LOSS iff xor of (h mod 3) == 0


def test_subtract_full_2_32_properties():
    """Config 5 at full size: closed-form values on 4M sampled keys + the root."""
    ctx, n, rec = _solve(SUB, (8,))
    assert n == 1 << 32
    rng = np.random.default_rng(7)
    keys = rng.integers(0, 1 << 32, size=1 << 22, dtype=np.uint64)
    recs = ctx.query(keys)
    assert np.array_equal(recs >> 14, _closed_form_values(keys, 8))
    # remoteness: heaps of one kind only -> single-heap formula R(3k)=2k, R(3k+1)=R(3k+2)=2k+1
    for h in range(16):
        r1 = int(ctx.query([h])[0]) & 0x3FFF
        assert r1 == (2 * (h // 3) + (0 if h % 3 == 0 else 1))
    assert rec >> 14 == 1               # all heaps 15: xor of (15 mod 3) = 0 -> LOSS


def test_subtract_8_heaps_full_table_vs_oracle(oracle):
    """Config 5 at FULL size: the 2^32 table of the headline kernel instance (the box
    engine's box_tier_kernel, csrc/dense_box.hip, the 8-heap default) equals the C
    oracle's, through the order-independent
    digest of every (key, record) -- against the committed oracle digest
    (tests/golden/make_oracle_digests.py) and a live oracle solve on the host.
    Semantics: reference src/new_process.py:189-198, 249-250."""
    ref = json.load(open(os.path.join(GOLDEN, "oracle_digests.json")))["subtract_8"]
    ctx, n, rec = _solve(SUB, (8,))
    got = ctx.digest()
    assert (n, rec) == (ref["positions"], ref["root_record"])
    assert got == (ref["digest"], ref["positions"])
    ctx.close()
    live = oracle.subtract_dense_mt(8)
    assert oracle.dense_digest(live) == got[0]
    assert int(live[-1]) == rec


def test_subtract_7_heaps_vs_oracle_digest(oracle):
    ref = oracle.subtract_dense(7)
    ctx, n, rec = _solve(SUB, (7,))
    keys = np.arange(1 << 28, dtype=np.uint64)
    assert ctx.digest() == (digest(keys, ref), 1 << 28)


def test_plugins_route_to_device():
    """Our plugin modules are matched to descriptors and solved on the device."""
    root_lines = json.load(open(os.path.join(GOLDEN, "roots.json")))
    for rel, attrs, expect in [
        ("test_games/mttt.py", {}, root_lines["mttt/blank"]["canonical"]),
        ("test_games/tic_tac_toe_np.py", {}, "TIE in 9 moves"),
        ("test_games/four_to_one.py", {}, "WIN in 3 moves"),
        ("test_games/othello_bit_new.py", {"length": 4, "height": 4}, "LOSS in 12 moves"),
        ("test_games/toot_and_otto_bitstring.py", {"length": 4, "height": 3}, "TIE in 12 moves"),
    ]:
        mod = load_plugin(rel, **attrs)
        s = Solver(mod, device=0)
        s.solve()
        assert s.root_line() == expect, rel


@pytest.mark.slow
def test_toot_6x4_known_per_ply_counts():
    """Config 3 at full size: per-ply reachable counts = SURVEY Appendix D."""
    app_d = [1, 12, 114, 748, 4266, 19692, 81140, 285708, 928196, 2665424, 7098172, 17010952,
             37792450, 64636776, 100084356, 136321692, 169785424, 180777508, 172831136,
             135153280, 91440950, 45953432, 19196602, 4537828, 606968]
    ctx, n, rec = _solve(TOOT, (6, 4))
    assert n == 1187212827
    assert [int(x) for x in ctx.tier_counts()] == app_d


@pytest.mark.parametrize("board", ["toot_4x4", "toot_5x4", "toot_6x4"])
@pytest.mark.parametrize("ranks", [1, 8])
def test_toot_large_boards_vs_oracle_digest(board, ranks):
    """Toot 4x4 / 5x4 / 6x4 (3.5 M / 70 M / 1.19 G positions; 6x4 is config 3):
    per-ply counts, root record and the full-table digest equal the C oracle's
    (tests/golden/make_oracle_digests.py), on one GPU and hash-sharded over 8
    loopback ranks.  Rules: reference test_games/toot_and_otto_bitstring.py:46-115."""
    ref = json.load(open(os.path.join(GOLDEN, "oracle_digests.json")))[board]
    L, H = (int(v) for v in board.split("_")[1].split("x"))
    ctx = Context(TOOT, (L, H), device=0)
    if ranks > 1:
        ctx.set_option(_lib.OPT_VIRTUAL_RANKS, ranks)
    n, rec = ctx.solve(ctx.initial())
    assert n == ref["positions"] and rec == ref["root_record"]
    assert [int(x) for x in ctx.tier_counts()] == ref["per_ply"]
    assert ctx.digest() == (ref["digest"], ref["positions"])


def _toot_mirror(k, L, H):
    """Left-right mirror of a Toot key (planes at bits 16 and 16 + L*H, cell L*y + x)."""
    A = L * H

    def plane(p):
        return sum(((p >> (L * y + x)) & 1) << (L * y + L - 1 - x) for y in range(H) for x in range(L))

    return (k & 0xFFFF) | (plane((k >> 16) & ((1 << A) - 1)) << 16) | (plane((k >> (A + 16)) & ((1 << A) - 1)) << (A + 16))


@pytest.mark.parametrize("board", ["toot_4x4", "toot_5x4"])
@pytest.mark.parametrize("ranks", [1, 8])
def test_toot_symmetry_off_matches_oracle_and_halves_tables(board, ranks):
    """GM_OPT_SYMMETRY: with the mirror reduction off the solve gives the
    same oracle digest; on (the default) it stores about half the positions (the tables
    are sized from predicted insert counts, so their bytes shrink a little less)."""
    ref = json.load(open(os.path.join(GOLDEN, "oracle_digests.json")))[board]
    L, H = (int(v) for v in board.split("_")[1].split("x"))
    bytes_ = {}
    for sym in (0, 1):
        ctx = Context(TOOT, (L, H), device=0)
        ctx.set_option(_lib.OPT_SYMMETRY, sym)
        if ranks > 1:
            ctx.set_option(_lib.OPT_VIRTUAL_RANKS, ranks)
        n, rec = ctx.solve(ctx.initial())
        assert n == ref["positions"] and rec == ref["root_record"]
        assert [int(x) for x in ctx.tier_counts()] == ref["per_ply"]
        assert ctx.digest() == (ref["digest"], ref["positions"])
        bytes_[sym] = ctx.stats()["table_bytes"]
        ctx.close()
    assert bytes_[1] < 0.8 * bytes_[0]


@pytest.mark.parametrize("ranks", [1, 8])
def test_othello_board_symmetry_on_off_matches_golden(ranks):
    """Othello 4x4 with the reduction by the board symmetries that fix the root (games.hpp
    DescOthello::sym; from the start: rotation by 180, transpose, anti-transpose): the same
    golden table, digest and per-tier counts as without it, at one GPU and 8 loopback
    ranks, with about a quarter of the edges expanded."""
    keys, recs = golden("othello_4x4")
    edges, tiers = {}, {}
    for sym in (0, 1):
        ctx = Context(OTH, (4, 4), device=0)
        ctx.set_option(_lib.OPT_SYMMETRY, sym)
        if ranks > 1:
            ctx.set_option(_lib.OPT_VIRTUAL_RANKS, ranks)
        for _ in range(2):   # the second solve is a replay on one GPU
            n, rec = ctx.solve(ctx.initial())
            k, r = ctx.export()
            assert n == len(keys) and np.array_equal(k, keys) and np.array_equal(r, recs)
            assert ctx.digest() == (digest(keys, recs), len(keys))
            assert ctx.query(keys[::97]).tolist() == recs[::97].tolist()
        edges[sym] = ctx.stats()["n_edges"]
        tiers[sym] = [int(x) for x in ctx.tier_counts()]
        ctx.close()
    assert tiers[0] == tiers[1] and sum(tiers[1]) == len(keys)
    if ranks == 1:
        assert edges[1] < 0.4 * edges[0], edges


@pytest.mark.parametrize("ranks", [1, 3])
def test_toot_symmetry_custom_roots_vs_oracle(oracle, ranks):
    """Roots other than the empty board (Toot 4x3): a mirror-symmetric grandchild keeps the
    reduction on, an asymmetric child turns it off; both tables equal the C oracle's,
    mirror images included, and queries of mirror images agree."""
    hd = games.HostDescriptor(games.TootCodec(4, 3))
    root = hd.initial()
    _, kids, _ = hd.expand(root)
    grand = [g for k in kids for g in hd.expand(k)[1]]
    sym_root = next(g for g in grand if _toot_mirror(g, 4, 3) == g)
    asym_root = next(k for k in kids if _toot_mirror(k, 4, 3) != k)
    hd.close()
    for r in (sym_root, asym_root):
        ok, orec = oracle.solve(TOOT, (4, 3), root=r)
        ctx = Context(TOOT, (4, 3), device=0)
        if ranks > 1:
            ctx.set_option(_lib.OPT_VIRTUAL_RANKS, ranks)
        n, rec = ctx.solve(r)
        k, rr = ctx.export()
        assert n == len(ok) and np.array_equal(k, ok) and np.array_equal(rr, orec)
        mk = np.array([_toot_mirror(int(x), 4, 3) for x in ok[:2000]], dtype=np.uint64)
        if r == sym_root:
            assert np.array_equal(ctx.query(mk), ctx.query(ok[:2000]))
        ctx.close()


@pytest.mark.parametrize("ranks", [1, 8])
def test_toot_full_table_rerun(monkeypatch, ranks):
    """A pinned, far too small distinct-child prediction fills every large tier
    table: the insert pass must flag it and re-run into a larger table, and the
    solve must still equal the C oracle's digest (Toot 4x4)."""
    ref = json.load(open(os.path.join(GOLDEN, "oracle_digests.json")))["toot_4x4"]
    monkeypatch.setenv("GM_TEST_DEDUP_RATIO", "0.02")
    ctx = Context(TOOT, (4, 4), device=0)
    if ranks > 1:
        ctx.set_option(_lib.OPT_VIRTUAL_RANKS, ranks)
    n, rec = ctx.solve(ctx.initial())
    assert n == ref["positions"] and rec == ref["root_record"]
    assert [int(x) for x in ctx.tier_counts()] == ref["per_ply"]
    assert ctx.digest() == (ref["digest"], ref["positions"])
