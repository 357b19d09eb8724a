"""Explicit-graph engine (GM_GAME_GRAPH, gamesmanmpi_amd/graph.py): plugins no
device descriptor reproduces are enumerated on the host with their own functions
and resolved on the device.  CPU tests check the enumeration; GPU tests check the
solve against the golden tables and the canonical oracle (oracle/canonical.py)."""
import os

import numpy as np
import pytest

from conftest import REPO, golden, load_plugin
from gamesmanmpi_amd import games
from gamesmanmpi_amd.graph import enumerate_graph, position_key

import canonical


def test_enumeration_matches_golden_position_set():
    mod = load_plugin("test_games/mttt.py")
    positions, prim, off, kids = enumerate_graph(mod, mod.initial_position())
    keys, _ = golden("ttt")
    codec = games.TTTStringCodec()
    assert sorted(codec.key(p) for p in positions) == keys.tolist()
    assert len(off) == len(positions) + 1 and off[-1] == len(kids)
    assert all((prim[i] == 4) == (off[i + 1] > off[i]) for i in range(len(positions)))


def test_enumeration_numpy_boards():
    mod = load_plugin("test_games/tic_tac_toe_np.py")
    positions, prim, off, kids = enumerate_graph(mod, mod.initial_position())
    assert len(positions) == 5478 and len({position_key(p) for p in positions}) == 5478


def test_descriptorless_plugins_are_not_identified():
    for rel in ("tests/plugins/nim3.py", "tests/plugins/misere_ttt.py"):
        assert games.identify(load_plugin(rel)) is None


def _graph_solver(rel, **attrs):
    from gamesmanmpi_amd import Solver
    mod = load_plugin(rel, **attrs)
    s = Solver(mod, device=0, graph=True)
    s.solve()
    return mod, s


@pytest.mark.gpu
@pytest.mark.parametrize("rel,attrs,name,codec", [
    ("test_games/mttt.py", {}, "ttt", games.TTTStringCodec()),
    ("test_games/tic_tac_toe_np.py", {}, "ttt_np", games.TTTNumpyCodec()),
    ("test_games/four_to_one.py", {}, "four_to_one_four", games.FourToOneCodec()),
    ("test_games/othello_bit_new.py", {"length": 4, "height": 4}, "othello_4x4", games.OthelloCodec(4, 4)),
    ("test_games/toot_and_otto_bitstring.py", {"length": 3, "height": 3}, "toot_3x3", games.TootCodec(3, 3)),
])
def test_graph_engine_matches_golden(rel, attrs, name, codec):
    mod, s = _graph_solver(rel, **attrs)
    keys, recs = golden(name)
    idx, r = s.table()
    assert s.ctx.stats()["engine"] == 5 and len(idx) == len(keys)
    got = dict(zip((codec.key(s.codec.pos(i)) for i in idx.tolist()), r.tolist()))
    assert got == dict(zip(keys.tolist(), recs.tolist()))
    s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("rel", ["tests/plugins/nim3.py", "tests/plugins/misere_ttt.py"])
def test_graph_engine_matches_canonical_oracle_on_new_plugins(rel):
    from gamesmanmpi_amd import Solver
    mod = load_plugin(rel)
    table, positions = canonical.solve(mod)
    s = Solver(mod, device=0)           # auto: no descriptor -> explicit graph
    n, rec = s.solve()
    assert n == len(table)
    idx, r = s.table()
    for i, rr in zip(idx.tolist(), r.tolist()):
        v, rem = table[canonical.default_key(s.codec.pos(i))]
        assert (rr >> 14, rr & 0x3FFF) == (v, rem)
    assert s.root_line() == canonical.root_line(*table[canonical.default_key(mod.initial_position())])
    s.close()


@pytest.mark.gpu
def test_graph_engine_rejects_a_cycle():
    from gamesmanmpi_amd import Context, GMError, _lib
    ctx = Context(_lib.GAME_GRAPH, (), device=0)
    with pytest.raises(GMError, match="cycle"):
        ctx.solve_graph([4, 4], [0, 1, 2], [1, 0])


@pytest.mark.gpu
def test_launcher_solves_a_descriptorless_plugin(tmp_path):
    import io
    import solver_launcher
    out = io.StringIO()
    args = solver_launcher.build_parser().parse_args([os.path.join(REPO, "tests/plugins/nim3.py"),
                                                      "-sd", str(tmp_path)])
    assert solver_launcher.run(args, out=out) == 0
    mod = load_plugin("tests/plugins/nim3.py")
    table, _ = canonical.solve(mod)
    assert out.getvalue() == canonical.root_line(*table[mod.initial_position()]) + "\n"
    from gamesmanmpi_amd.persist import read_reference_tables
    back = read_reference_tables(str(tmp_path))
    assert back[str((5, 6, 7))] == table[(5, 6, 7)]
