"""Othello on the reference's default 8x8 board ON THE DEVICE (SURVEY
§8f.3): the reference plugin's 144-bit positions bind to the 128-bit-key descriptor
(csrc/games.hpp DescOthello8) and are solved by the hash-sharded sparse engine with 32-byte
table slots (csrc/sparse_tables.hpp WSlot), from endgame roots of the seed-5 playout
(tests/plugins/othello8_endgame.py).

* 10 empties (56,552 positions): every record equals the golden table the REFERENCE's plugin
  gives (tests/golden/othello_8x8_endgame.npz, keys = blake2b-8 of the position string), and
  the root line equals the canonical one -- on one GPU and on 8 virtual ranks;
* 12 empties (1.2 M positions): every record equals the explicit-graph path's (the plugin's
  own functions on the host, tests/test_graph.py pins that path at 10 empties).
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden, load_plugin

pytestmark = pytest.mark.gpu

ROOT12 = "30380028503841784646bfd6afc6be000200"


def _blake(pos):
    return int.from_bytes(hashlib.blake2b(pos.encode("ISO-8859-1"), digest_size=8).digest(), "big")


def _table_by_pos(solver):
    from gamesmanmpi_amd import _lib
    keys, recs = solver.table()
    return {solver.codec.pos(_lib.words_to_int(w)): int(r) for w, r in zip(keys.tolist(), recs.tolist())}


def _endgame(monkeypatch, hexroot=None):
    if hexroot:
        monkeypatch.setenv("GM_OTHELLO8_ROOT", hexroot)
    return load_plugin("tests/plugins/othello8_endgame.py")


@pytest.mark.parametrize("ranks", [1, 8])
def test_othello8_endgame_10_on_device_vs_reference_golden(monkeypatch, ranks):
    from gamesmanmpi_amd import Solver, _lib
    mod = _endgame(monkeypatch)
    s = Solver(mod, device=0)
    assert s.codec.params == (8, 8) and s.ctx.words == 3
    if ranks > 1:
        s.ctx.set_option(_lib.OPT_VIRTUAL_RANKS, ranks)
    n, rec = s.solve()
    st = s.ctx.stats()
    assert st["engine"] == _lib.ENGINE_DIST_SPARSE and st["world"] == ranks
    keys, recs = golden("othello_8x8_endgame")
    assert n == len(keys) == 56552
    got = {_blake(p): r for p, r in _table_by_pos(s).items()}
    assert got == dict(zip(keys.tolist(), recs.tolist()))
    roots = json.load(open(os.path.join(GOLDEN, "roots.json")))
    assert s.root_line() == roots["othello_8x8_endgame"]["canonical"]
    # lookups: every exported key answers its record; a key outside the solve answers 0xFFFF
    k, r = s.table()
    pick = np.arange(0, len(k), 97)
    assert np.array_equal(s.ctx.query(k[pick]), r[pick])
    start = s.ctx.initial()
    assert s.ctx.query([start])[0] == _lib.REC_UNSOLVED
    s.close()


def test_othello8_virtual_ranks_digest_equals_one_gpu(monkeypatch):
    """The hash partition changes nothing: 1, 3 and 8 virtual ranks give one digest."""
    from gamesmanmpi_amd import Solver, _lib
    mod = _endgame(monkeypatch)
    digests = []
    for ranks in (1, 3, 8):
        s = Solver(mod, device=0)
        if ranks > 1:
            s.ctx.set_option(_lib.OPT_VIRTUAL_RANKS, ranks)
        s.solve()
        digests.append(s.ctx.digest())
        assert (ranks == 1) == (s.ctx.stats()["exchanged_bytes"] == 0)
        s.close()
    assert digests[0] == digests[1] == digests[2] and digests[0][1] == 56552


def test_othello8_endgame_12_device_vs_graph_path():
    """12 empties (1.2 M positions): the plugin at its default 8x8 with the root passed as a
    custom position (solver_launcher.py --custom) binds the descriptor by its code fingerprint,
    and the device table equals the explicit-graph path's record for record (position strings
    of the plugin).  (The fingerprint covers the rule functions, not initial_position, so the
    launcher's --custom root keeps the binding: tests/test_abi.py
    ::test_launcher_custom_root_keeps_the_fingerprint_binding.)"""
    from gamesmanmpi_amd import Solver, _lib
    mod = load_plugin("test_games/othello_bit_new.py")
    root = bytes.fromhex(ROOT12).decode("latin-1")
    s = Solver(mod, root=root, device=0)
    assert s.ctx.words == 3
    n, rec = s.solve()
    assert s.ctx.stats()["engine"] == _lib.ENGINE_DIST_SPARSE
    dev = _table_by_pos(s)
    s.close()
    g = Solver(mod, root=root, device=0, graph=True)
    gn, grec = g.solve()
    idx, r = g.table()
    ref = {g.codec.pos(i): int(x) for i, x in zip(idx.tolist(), r.tolist())}
    g.close()
    assert n == gn == len(dev) == len(ref) and rec == grec
    assert dev == ref


def _empties(p):
    b = p.encode("latin-1")
    return 64 - bin(int.from_bytes(b[0:8], "big") | int.from_bytes(b[8:16], "big")).count("1")


def test_othello8_edge_roots_vs_canonical():
    """Edge roots on the device path, each table equal to the canonical oracle over the plugin
    (oracle/canonical.py): a full board (primitive: one position), a board with one empty
    square, and a position of at most 10 empties whose mover must pass (the pass keeps the
    mover, othello_bit_new.py:122-124; a second pass ends the game, :82)."""
    import random
    from gamesmanmpi_amd import Solver
    import canonical
    mod = load_plugin("test_games/othello_bit_new.py")
    rng = random.Random(11)
    found = {}
    for _ in range(400):
        p = mod.initial_position()
        while mod.primitive(p) == 4:
            ms = mod.gen_moves(p)
            if ms == [None] and _empties(p) <= 10:
                found.setdefault("pass", p)
            if _empties(p) == 1:
                found.setdefault("one_empty", p)
            p = mod.do_move(p, ms[rng.randrange(len(ms))])
        if _empties(p) == 0:
            found.setdefault("full", p)
        if len(found) == 3:
            break
    assert set(found) == {"pass", "one_empty", "full"}, found.keys()
    for name, root in found.items():
        s = Solver(mod, root=root, device=0)
        n, rec = s.solve()
        dev = _table_by_pos(s)
        s.close()
        table, positions = canonical.solve(mod, root)
        ref = {positions[k]: (v << 14) | r for k, (v, r) in table.items()}
        assert n == len(ref) and dev == ref, name
