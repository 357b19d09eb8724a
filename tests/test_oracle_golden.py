"""The oracle is pinned: C and Python restatements reproduce the golden fixtures.

The fixtures (tests/golden/*.npz, roots.json) were generated from the REFERENCE's
own plugin modules by tests/golden/make_golden.py; live.json records that the
reference's live engine (src/new_process.py) agrees with them on every value.
"""
import json
import os

import numpy as np
import pytest

import canonical
from conftest import GOLDEN, digest, golden, load_plugin

F2O, TTT, TOOT, OTH, SUB = 1, 2, 3, 4, 5

CASES = [
    ("ttt", TTT, (), None),
    ("othello_4x4", OTH, (4, 4), None),
    ("toot_3x3", TOOT, (3, 3), None),
    ("toot_4x3", TOOT, (4, 3), None),
    ("four_to_one_four", F2O, (), 4),
    ("four_to_one_six", F2O, (), 6),
    ("four_to_one_one", F2O, (), 1),
    ("four_to_one_zero", F2O, (), 0),
]


@pytest.mark.parametrize("name,game,params,root", CASES)
def test_c_oracle_matches_golden(oracle, name, game, params, root):
    keys, recs = golden(name)
    k, r = oracle.solve(game, params, root)
    assert np.array_equal(k, keys)
    assert np.array_equal(r, recs)


def test_golden_summary_counts():
    # SURVEY Appendix C probe numbers
    for name, (w, l, t) in {"ttt": (2836, 1574, 1068), "othello_4x4": (24481, 24069, 5539),
                            "toot_4x3": (36057, 15393, 148677), "toot_3x3": (0, 0, 11097)}.items():
        v = golden(name)[1] >> 14
        assert ((v == 0).sum(), (v == 1).sum(), (v == 2).sum()) == (w, l, t)


def test_reference_root_expectations():
    roots = json.load(open(os.path.join(GOLDEN, "roots.json")))
    agree = [k for k, v in roots.items() if "reference_test_expects" in v
             and v["canonical"] == v["reference_test_expects"]]
    # 8 of the reference's 9 game_tests agree with the canonical semantics; one_row's
    # expectation (mttt_test.py:61-71, TIE in 3) is wrong under every reference path.
    assert len(agree) == 8
    assert roots["mttt/one_row"]["canonical"] == "WIN in 5 moves"
    assert roots["othello_4x4"]["canonical"] == "LOSS in 12 moves"
    assert roots["toot_4x3"]["canonical"] == "TIE in 12 moves"


def test_live_reference_engine_agrees_on_values():
    live = json.load(open(os.path.join(GOLDEN, "live.json")))
    for case, v in live.items():
        assert v["value_mismatches"] == 0, case
        assert v["positions_live"] == v["positions_canonical"], case
        # its remoteness is only ever one short
        assert set(v["remoteness_deltas"]) <= {"-1"}, case


def _key_mttt(pos):
    return sum({"_": 0, "X": 1, "O": 2}[c] * 3 ** i for i, c in enumerate(pos))


def test_python_canonical_on_our_mttt_plugin():
    mod = load_plugin("test_games/mttt.py")
    table, positions = canonical.solve(mod)
    keys, recs = golden("ttt")
    got = sorted((_key_mttt(positions[k]), (v << 14) | r) for k, (v, r) in table.items())
    assert [g[0] for g in got] == keys.tolist()
    assert [g[1] for g in got] == recs.tolist()


def test_python_canonical_on_our_ttt_numpy_plugin():
    mod = load_plugin("test_games/tic_tac_toe_np.py")
    table, positions = canonical.solve(mod)
    keys, recs = golden("ttt_np")
    got = sorted((sum(int(positions[k][x][y]) * 3 ** (x + 3 * y) for x in range(3) for y in range(3)),
                  (v << 14) | r) for k, (v, r) in table.items())
    assert [g[0] for g in got] == keys.tolist()
    assert [g[1] for g in got] == recs.tolist()


@pytest.mark.parametrize("root,name", [("4", "four"), ("6", "six"), ("1", "one"), ("0", "zero")])
def test_python_canonical_on_our_four_to_one_plugin(root, name):
    mod = load_plugin("test_games/four_to_one.py")
    table, positions = canonical.solve(mod, root)
    keys, recs = golden("four_to_one_" + name)
    got = sorted((int(positions[k]) & (2 ** 64 - 1), (v << 14) | r) for k, (v, r) in table.items())
    assert [g[0] for g in got] == keys.tolist()
    assert [g[1] for g in got] == recs.tolist()


def _bits_key(nkeep):
    def k(pos):
        raw = pos.encode("ISO-8859-1")
        return int.from_bytes(raw, "big") >> (8 * len(raw) - nkeep)
    return k


@pytest.mark.parametrize("plugin,dims,name,nkeep", [
    ("test_games/othello_bit_new.py", (4, 4), "othello_4x4", 48),
    ("test_games/toot_and_otto_bitstring.py", (3, 3), "toot_3x3", 34),
])
def test_python_canonical_on_our_bitboard_plugins(plugin, dims, name, nkeep):
    mod = load_plugin(plugin, length=dims[0], height=dims[1])
    table, positions = canonical.solve(mod)
    keys, recs = golden(name)
    kf = _bits_key(nkeep)
    got = sorted((kf(positions[k]), (v << 14) | r) for k, (v, r) in table.items())
    assert [g[0] for g in got] == keys.tolist()
    assert [g[1] for g in got] == recs.tolist()


def _blake8(pos):
    import hashlib
    return int.from_bytes(hashlib.blake2b(pos.encode("ISO-8859-1"), digest_size=8).digest(), "big")


def test_python_canonical_on_our_othello_8x8_endgame():
    """§8f.3 at the reference's own 8x8 board: our plugin (test_games/othello_bit_new.py at its
    default 8x8) from the endgame root of tests/plugins/othello8_endgame.py gives, under the
    canonical oracle, exactly the golden table made from the REFERENCE's plugin (positions
    keyed by an 8-byte blake2b of their 144-bit string).  It binds the 128-bit-key descriptor,
    whose device tables tests/test_gpu_othello8.py checks against the same golden table."""
    from gamesmanmpi_amd import games
    mod = load_plugin("tests/plugins/othello8_endgame.py")
    c = games.identify(mod)
    assert c is not None and c.params == (8, 8)
    table, positions = canonical.solve(mod)
    keys, recs = golden("othello_8x8_endgame")
    got = sorted((_blake8(positions[k]), (v << 14) | r) for k, (v, r) in table.items())
    assert [g[0] for g in got] == keys.tolist()
    assert [g[1] for g in got] == recs.tolist()


def test_subtract_oracle_closed_form_and_f2o(oracle):
    # values: LOSS iff xor_i (h_i mod 3) == 0; one heap == Four-To-One (golden) for piles >= 0
    rec = oracle.subtract_dense(4)
    keys = np.arange(1 << 16, dtype=np.uint64)
    g = np.zeros(len(keys), dtype=np.int64)
    for i in range(4):
        g ^= ((keys >> np.uint64(4 * i)) & np.uint64(15)).astype(np.int64) % 3
    assert np.array_equal(rec >> 14, np.where(g == 0, 1, 0))
    one = oracle.subtract_dense(1)
    fk, fr = golden("four_to_one_six")
    for k, r in zip(fk.tolist(), fr.tolist()):
        if k < 16:
            assert one[k] == r


def test_subtract_dense_equals_generic_oracle(oracle):
    dense = oracle.subtract_dense(3)
    k, r = oracle.solve(SUB, (3,))
    assert np.array_equal(k, np.arange(4096, dtype=np.uint64)) and np.array_equal(r, dense)


@pytest.mark.parametrize("heaps", [1, 2, 3, 4, 5, 6])
def test_subtract_dense_multithreaded_equals_sequential(oracle, heaps):
    # the bench's multi-core cpu_baseline must compute the same table
    assert np.array_equal(oracle.subtract_dense_mt(heaps, 4), oracle.subtract_dense(heaps))


def test_subtract_plugin_canonical(oracle):
    mod = load_plugin("test_games/subtraction.py", HEAPS=2)
    table, positions = canonical.solve(mod)
    k, r = oracle.solve(SUB, (2,))
    got = sorted((positions[key], (v << 14) | rr) for key, (v, rr) in table.items())
    assert [g[0] for g in got] == k.tolist() and [g[1] for g in got] == r.tolist()


def test_toot_4x4_oracle_totals(oracle):
    # 4x4 = 3,468,773 positions
    k, r = oracle.solve(TOOT, (4, 4))
    assert len(k) == 3468773
    assert (r != 0xFFFF).all()


# ---- the sorted-layer OpenMP oracle (oracle_solve_layered): the full-size checker
# of configs 3 and 4 and the bench's CPU baseline for them.  Pinned here to the
# same golden tables (digest equality) and to the hash-map oracle.

@pytest.mark.parametrize("name,game,params,root", CASES)
def test_layered_oracle_matches_golden(oracle, name, game, params, root):
    keys, recs = golden(name)
    n, dg, rr, tiers = oracle.solve_layered(game, params, root)
    assert n == len(keys) and sum(tiers) == n
    assert dg == digest(keys, recs)
    root_key = oracle.initial(game, params) if root is None else root
    assert rr == int(recs[np.searchsorted(keys, np.uint64(root_key & (2 ** 64 - 1)))])


@pytest.mark.parametrize("threads", [1, 3, 0])
def test_layered_oracle_toot_4x4_equals_hash_oracle(oracle, threads):
    ref = json.load(open(os.path.join(GOLDEN, "oracle_digests.json")))["toot_4x4"]
    n, dg, rr, tiers = oracle.solve_layered(TOOT, (4, 4), threads=threads)
    assert (n, dg, rr, tiers) == (ref["positions"], ref["digest"], ref["root_record"], ref["per_ply"])


def test_layered_oracle_subtract_equals_dense(oracle):
    for heaps in (2, 3, 4):
        n, dg, rr, tiers = oracle.solve_layered(SUB, (heaps,))
        dense = oracle.subtract_dense(heaps)
        assert n == 16 ** heaps and dg == oracle.dense_digest(dense)
        assert dg == digest(np.arange(16 ** heaps, dtype=np.uint64), dense)
        assert rr == int(dense[-1])


def test_full_size_oracle_digests_committed():
    """tests/golden/oracle_digests.json holds the full-size oracle tables of configs 3-5
    (tests/golden/make_oracle_digests.py); its Toot 6x4 per-ply counts are SURVEY App. D."""
    ref = json.load(open(os.path.join(GOLDEN, "oracle_digests.json")))
    app_d = [1, 12, 114, 748, 4266, 19692, 81140, 285708, 928196, 2665424, 7098172, 17010952,
             37792450, 64636776, 100084356, 136321692, 169785424, 180777508, 172831136,
             135153280, 91440950, 45953432, 19196602, 4537828, 606968]
    assert ref["toot_6x4"]["per_ply"] == app_d and ref["toot_6x4"]["positions"] == sum(app_d) == 1187212827
    assert ref["subtract_8"]["positions"] == 1 << 32
    assert ref["subtract_8"]["root_record"] == (1 << 14) | 80        # LOSS in 80 (all heaps 15)
    keys, recs = golden("othello_4x4")
    assert ref["othello_4x4"]["digest"] == digest(keys, recs)
    assert ref["othello_4x4"]["root_record"] == (1 << 14) | 12       # LOSS in 12


def test_dense_digest_matches_python_formula(oracle):
    rng = np.random.default_rng(3)
    recs = rng.integers(0, 1 << 16, size=100003, dtype=np.uint16)
    assert oracle.dense_digest(recs) == digest(np.arange(len(recs), dtype=np.uint64), recs)


def test_othello_player_flip_maps_reachable_to_unreachable():
    """The reference's declared Othello symmetry, player_flip (othello_bit_new.py:224-235:
    every piece changes colour and the turn advances), merges no two reachable positions:
    a reachable position's mover is fixed by its piece count (a pass keeps the mover, who
    passes again and ends the game), and player_flip keeps the pieces but swaps the mover.
    So the device reduces Othello by the board symmetries that fix the root instead
    (DescOthello::sym); this pins the argument on the reference's own 54,089 positions."""
    keys, _ = golden("othello_4x4")
    A = 16
    ks = set(int(k) for k in keys)
    m = (1 << A) - 1
    for k in ks:
        w, b, turn, pas = (k >> (A + 16)) & m, (k >> 16) & m, (k >> 8) & 0xFF, k & 0xFF
        flipped = (b << (A + 16)) | (w << 16) | ((3 - turn) << 8) | pas
        assert flipped not in ks
        assert (bin(w | b).count("1") % 2 == 0) == (turn == 2)   # WHITE moves on an even piece count
