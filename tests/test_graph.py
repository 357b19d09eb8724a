"""Explicit-graph engine (GM_GAME_GRAPH, gamesmanmpi_amd/graph.py): plugins no
device descriptor reproduces are enumerated on the host with their own functions
and resolved on the device.  CPU tests check the enumeration; GPU tests check the
solve against the golden tables and the canonical oracle (oracle/canonical.py)."""
import os
import time

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
def test_graph_engine_othello_8x8_endgame_matches_golden():
    """Othello on the reference's default 8x8 board from an endgame root (10 empty squares,
    56,552 positions) through the explicit-graph path (host walk with the plugin's functions,
    GPU resolve; graph=True -- the plugin also binds the 128-bit-key descriptor,
    tests/test_gpu_othello8.py): every record equals the golden table of the REFERENCE's
    plugin from the same root."""
    import hashlib
    import json
    from conftest import GOLDEN
    from gamesmanmpi_amd import Solver
    mod = load_plugin("tests/plugins/othello8_endgame.py")
    s = Solver(mod, device=0, graph=True)
    n, rec = s.solve()
    keys, recs = golden("othello_8x8_endgame")
    assert s.ctx.stats()["engine"] == 5 and n == len(keys)
    idx, r = s.table()
    blake = [int.from_bytes(hashlib.blake2b(s.codec.pos(i).encode("ISO-8859-1"), digest_size=8).digest(), "big")
             for i in idx.tolist()]
    assert dict(zip(blake, r.tolist())) == dict(zip(keys.tolist(), recs.tolist()))
    roots = json.load(open(os.path.join(GOLDEN, "roots.json")))
    assert s.root_line() == roots["othello_8x8_endgame"]["canonical"]
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


@pytest.mark.parametrize("workers", [2, 3])
@pytest.mark.parametrize("rel", ["test_games/mttt.py", "test_games/tic_tac_toe_np.py", "tests/plugins/nim3.py",
                                 "test_games/four_to_one.py"])
def test_parallel_enumeration_equals_serial(monkeypatch, rel, workers):
    """The sharded walk (forced on with PAR_MIN = 8: worker processes own the positions
    by fingerprint, the parent numbers fingerprints with numpy) gives the serial walk's
    numbering, primitives and CSR exactly."""
    from gamesmanmpi_amd import graph
    mod = load_plugin(rel)
    root = mod.initial_position()
    serial = enumerate_graph(mod, root, workers=1)
    monkeypatch.setattr(graph, "PAR_MIN", 8)
    monkeypatch.setattr(graph, "PAR_START", 8)
    par = enumerate_graph(mod, root, workers=workers)
    assert [position_key(p) for p in par[0]] == [position_key(p) for p in serial[0]]
    for a, b in zip(par[1:], serial[1:]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("collide", ["first_level", "always"])
def test_parallel_numbering_survives_8_byte_fingerprint_collisions(monkeypatch, collide):
    """The parent compares fingerprints by their first 8 bytes and checks all 16; with
    the first 8 forced equal (as if two positions collided there) the level falls back to
    the whole 16 bytes -- before the walk goes parallel, or from its first parallel level
    -- and the numbering is still the serial walk's."""
    from gamesmanmpi_amd import graph
    mod = load_plugin("test_games/mttt.py")
    root = mod.initial_position()
    serial = enumerate_graph(mod, root, workers=1)
    real = graph._halves

    def halves(F):
        hi, lo = real(F)
        return np.zeros_like(hi) if collide == "always" or len(F) > 2000 else hi, lo
    monkeypatch.setattr(graph, "_halves", halves)
    monkeypatch.setattr(graph, "PAR_MIN", 8)
    monkeypatch.setattr(graph, "PAR_START", 8)
    par = enumerate_graph(mod, root, workers=2)
    assert [position_key(p) for p in par[0]] == [position_key(p) for p in serial[0]]
    for a, b in zip(par[1:], serial[1:]):
        assert np.array_equal(a, b)


def test_parallel_walk_with_declared_symmetry(monkeypatch):
    """The sharded walk on orbit representatives: the workers canonicalise children and
    count the orbit members of the positions they keep (765 orbits, 5,478 positions)."""
    from gamesmanmpi_amd import graph
    monkeypatch.setattr(graph, "PAR_MIN", 8)
    monkeypatch.setattr(graph, "PAR_START", 8)
    mod = load_plugin("tests/plugins/ttt_symmetric.py")
    ser = graph.GraphCodec(mod, mod.initial_position(), workers=1)
    par = graph.GraphCodec(mod, mod.initial_position(), workers=3)
    assert par.n_positions == ser.n_positions == 5478 and len(par.positions) == 765
    assert par.positions == ser.positions
    assert all(np.array_equal(a, b) for a, b in ((par.prim, ser.prim), (par.off, ser.off), (par.kids, ser.kids)))


def test_small_plugins_start_no_worker(monkeypatch):
    """a plugin whose levels stay small (tic-tac-toe: at most 1,520 positions
    per level) never starts the worker processes."""
    from gamesmanmpi_amd import graph
    def pool(*a):
        raise AssertionError("worker processes started for tic-tac-toe")
    monkeypatch.setattr(graph, "_ShardPool", pool)
    monkeypatch.setattr(graph, "_prestart", pool)
    mod = load_plugin("test_games/mttt.py")
    pos, prim, off, kids = graph.enumerate_graph(mod, mod.initial_position(), workers=8)
    assert len(pos) == 5478


def test_enumeration_fails_fast_with_a_projection():
    """Othello at its 8x8 default from the start, walked on the host: the walk stops with the
    level sizes and the projected next level once the projection passes the limit."""
    import time
    from gamesmanmpi_amd.graph import TooLarge
    mod = load_plugin("test_games/othello_bit_new.py")
    t = time.perf_counter()
    with pytest.raises(TooLarge, match="projected"):
        enumerate_graph(mod, mod.initial_position(), limit=20_000, workers=1)
    assert time.perf_counter() - t < 60


def test_parallel_walk_fails_fast_and_ends_its_workers(monkeypatch):
    """The projection stops a sharded walk too: TooLarge is raised from the parent's
    numbering while the workers run ahead, and the workers are ended (none outlives it)."""
    import multiprocessing as mp
    import time
    from gamesmanmpi_amd import graph
    monkeypatch.setattr(graph, "PAR_MIN", 64)
    monkeypatch.setattr(graph, "PAR_START", 64)
    mod = load_plugin("test_games/othello_bit_new.py")
    t = time.perf_counter()
    with pytest.raises(graph.TooLarge):
        enumerate_graph(mod, mod.initial_position(), limit=20_000, workers=3)
    assert time.perf_counter() - t < 60
    deadline = time.time() + 10
    while mp.active_children() and time.time() < deadline:
        time.sleep(0.05)
    assert not mp.active_children()


def test_parallel_walk_never_rebuilds_a_patched_plugin(monkeypatch):
    """Workers rebuild the plugin from its file; a caller-replaced function must keep the
    walk serial (else workers would expand the file's game), while a caller-changed table
    travels to the workers.  Either way the graph equals the serial walk's."""
    import gamesmanmpi_amd.graph as G
    monkeypatch.setattr(G, "PAR_MIN", 16)
    monkeypatch.setattr(G, "PAR_START", 16)
    mod = load_plugin("test_games/mttt.py")
    orig = mod.primitive
    mod.primitive = lambda pos: 1 if orig(pos) == 2 else orig(pos)   # misere: full board LOSS
    assert G._module_spec(mod) is None
    ser = enumerate_graph(mod, mod.initial_position(), workers=1)
    par = enumerate_graph(mod, mod.initial_position(), workers=3)
    assert ser[0] == par[0] and all(np.array_equal(a, b) for a, b in zip(ser[1:], par[1:]))
    assert (par[1] == 1).sum() > (enumerate_graph(load_plugin("test_games/mttt.py"), "_" * 9, workers=1)[1] == 1).sum()


def test_symmetry_functions_fixing_the_root_reduce_the_walk():
    """symmetry_functions() (the reference's hook, othello_bit_new.py:224-225): the graph
    walk keeps one representative per orbit of the declared functions that fix the root
    and stands for every member (tests/plugins/ttt_symmetric.py: 765 orbits of 5,478
    positions); functions that move the root are not used."""
    from gamesmanmpi_amd.graph import GraphCodec, symmetry_generators
    mod = load_plugin("tests/plugins/ttt_symmetric.py")
    c = GraphCodec(mod, mod.initial_position(), workers=1)
    assert c.symmetry == [0, 1] and len(c.positions) == 765 and c.n_positions == 5478
    members = [p for i in range(len(c.positions)) for p in c.members(i)]
    assert len(members) == len(set(members)) == 5478
    table, _ = canonical.solve(load_plugin("test_games/mttt.py"))
    assert set(members) == set(table)
    assert all(c.key(p) == c.key(mod.rotate(p)) for p in members[:500])
    assert symmetry_generators(mod, "X___O____") == []      # neither generator fixes it
    oth = load_plugin("test_games/othello_bit_new.py", length=4, height=4)
    assert not hasattr(oth, "symmetry_functions") or symmetry_generators(oth, oth.initial_position()) == []


@pytest.mark.gpu
def test_graph_engine_with_declared_symmetry_matches_golden(tmp_path):
    """The symmetric plugin solved through the graph engine (765 orbits on the device):
    every member's record equals the golden mttt table; -sd writes all 5,478 positions."""
    import io
    import solver_launcher
    from gamesmanmpi_amd import Solver
    mod = load_plugin("tests/plugins/ttt_symmetric.py")
    s = Solver(mod, device=0, graph=True)
    n, rec = s.solve()
    keys, recs = golden("ttt")
    want = dict(zip(keys.tolist(), recs.tolist()))
    codec = games.TTTStringCodec()
    idx, r = s.table()
    assert n == 5478 and len(idx) == 765
    got = {codec.key(p): rr for i, rr in zip(idx.tolist(), r.tolist()) for p in s.codec.members(i)}
    assert got == want
    assert s.lookup("XO_______") == (want[codec.key("XO_______")] >> 14, want[codec.key("XO_______")] & 0x3FFF)
    s.close()
    out = io.StringIO()
    args = solver_launcher.build_parser().parse_args([os.path.join(REPO, "tests/plugins/ttt_symmetric.py"),
                                                      "-sd", str(tmp_path)])
    assert solver_launcher.run(args, out=out) == 0 and out.getvalue() == "TIE in 9 moves\n"
    from gamesmanmpi_amd.persist import read_reference_tables
    back = read_reference_tables(str(tmp_path))
    assert len(back) == 5478 and back["X________"] == (want[1] >> 14, want[1] & 0x3FFF)


def test_worker_mesh_drops_unauthenticated_connections():
    """The workers' mesh (walk_worker._mesh) listens on abstract unix sockets, whose names
    any local process can list; a connection without the walk's key is refused and the
    mesh still forms."""
    import threading
    from multiprocessing import AuthenticationError
    from multiprocessing.connection import Client
    from gamesmanmpi_amd import walk_worker

    tag, key, nw = "gm-walk-test-%d-%s" % (os.getpid(), os.urandom(4).hex()), os.urandom(32), 3
    out, errs = [None] * nw, []

    def run(w):
        try:
            out[w] = walk_worker._mesh(w, nw, tag, key, timeout_s=30.0)
        except BaseException as e:   # pragma: no cover - reported below
            errs.append(e)

    # a rogue client first: worker 0's listener must exist before it can connect
    th = [threading.Thread(target=run, args=(0,))]
    th[0].start()
    rogue = None
    for _ in range(2000):
        try:
            with pytest.raises(AuthenticationError):
                Client("\0%s-0" % tag, family="AF_UNIX", authkey=b"wrong key")
            rogue = True
            break
        except (FileNotFoundError, ConnectionRefusedError):
            import time
            time.sleep(0.005)
    assert rogue
    for w in range(1, nw):
        th.append(threading.Thread(target=run, args=(w,)))
        th[-1].start()
    for t in th:
        t.join(60)
    assert not errs
    for w in range(nw):
        for p in range(nw):
            if p != w:
                out[w][p].send_bytes(b"%d>%d" % (w, p))
    for w in range(nw):
        for p in range(nw):
            if p != w:
                assert out[w][p].recv_bytes() == b"%d>%d" % (p, w)


def _silent_stranger(tag, me):
    import socket
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    for _ in range(500):
        try:
            s.connect("\0" + tag + "-%d" % me)
            return s
        except (FileNotFoundError, ConnectionRefusedError):
            time.sleep(0.01)
    raise AssertionError("worker socket never appeared")


def test_walk_mesh_survives_a_silent_connection_and_times_out():
    """a local process that connects to a walk worker's socket and never answers
    the HMAC challenge is dropped after the handshake limit (the mesh still forms with the
    real peer), and a peer that never connects ends the mesh with TimeoutError instead of a
    hang (walk_worker._mesh)."""
    import os
    import threading
    from gamesmanmpi_amd import walk_worker
    old = walk_worker.HANDSHAKE_S
    walk_worker.HANDSHAKE_S = 1.0
    try:
        key, tag = os.urandom(32), "gmtest-%d" % os.getpid()
        got = {}
        t0 = threading.Thread(target=lambda: got.update(w0=walk_worker._mesh(0, 2, tag, key, timeout_s=20)))
        t0.start()
        stranger = _silent_stranger(tag, 0)
        time.sleep(0.1)
        peers1 = walk_worker._mesh(1, 2, tag, key, timeout_s=20)
        t0.join(30)
        assert not t0.is_alive() and got["w0"][1] is not None and peers1[0] is not None
        got["w0"][1].send_bytes(b"ping")
        assert peers1[0].recv_bytes() == b"ping"
        stranger.close()
        tag2 = tag + "b"
        err = {}

        def lone():
            try:
                walk_worker._mesh(0, 2, tag2, key, timeout_s=2.5)
            except Exception as e:   # noqa: BLE001 -- the test inspects it
                err["e"] = e
        t = time.time()
        th = threading.Thread(target=lone)
        th.start()
        s2 = _silent_stranger(tag2, 0)
        th.join(30)
        assert isinstance(err.get("e"), TimeoutError) and time.time() - t < 10
        s2.close()
    finally:
        walk_worker.HANDSHAKE_S = old


def test_walk_mesh_connecting_side_times_out_on_a_silent_acceptor():
    """the CONNECTING side is bounded too -- a lower-numbered 'peer' that accepts
    the connection and never sends the HMAC challenge ends worker 1's mesh with TimeoutError
    within the handshake limit instead of blocking in the challenge exchange."""
    import os
    import socket
    from gamesmanmpi_amd import walk_worker
    old = walk_worker.HANDSHAKE_S
    walk_worker.HANDSHAKE_S = 1.0
    tag = "gmtest-acc-%d-%s" % (os.getpid(), os.urandom(3).hex())
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    srv.bind("\0" + tag + "-0")
    srv.listen(4)
    try:
        t = time.time()
        with pytest.raises(TimeoutError):
            walk_worker._mesh(1, 2, tag, os.urandom(32), timeout_s=20)
        assert time.time() - t < 10
    finally:
        walk_worker.HANDSHAKE_S = old
        srv.close()
