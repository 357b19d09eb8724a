"""The drop-in CLIs: the reference's 9 game_tests re-expressed (game_tests/*.py).

The reference compares the launcher's exact stdout line for Four-To-One roots 4/6/1/0
(four_to_one_test.py:14-59) and five mttt roots (mttt_test.py:14-71).  Expectations
here are the canonical ones (roots.json); they equal the reference's for 8 of 9,
and one_row is WIN in 5 (the reference test's "TIE in 3" holds under no reference
engine path).
"""
import io
import json
import os

import pytest

from conftest import GOLDEN, REPO

import solver_launcher
import solve_local

ROOTS = json.load(open(os.path.join(GOLDEN, "roots.json")))

CASES = [
    (["test_games/four_to_one.py"], "four_to_one/four"),
    (["test_games/four_to_one.py", "--init_pos", "six", "--custom", "tests/custom/four_to_one_roots.py"],
     "four_to_one/six"),
    (["test_games/four_to_one.py", "--init_pos", "one", "--custom", "tests/custom/four_to_one_roots.py"],
     "four_to_one/one"),
    (["test_games/four_to_one.py", "--init_pos", "zero", "--custom", "tests/custom/four_to_one_roots.py"],
     "four_to_one/zero"),
    (["test_games/mttt.py"], "mttt/blank"),
    (["test_games/mttt.py", "--init_pos", "tie_in_one", "--custom", "tests/custom/mttt_roots.py"],
     "mttt/tie_in_one"),
    (["test_games/mttt.py", "--init_pos", "win_in_one", "--custom", "tests/custom/mttt_roots.py"],
     "mttt/win_in_one"),
    (["test_games/mttt.py", "--init_pos", "side_columns", "--custom", "tests/custom/mttt_roots.py"],
     "mttt/side_columns"),
    (["test_games/mttt.py", "--init_pos", "one_row", "--custom", "tests/custom/mttt_roots.py"],
     "mttt/one_row"),
]


def _abs(argv):
    return [os.path.join(REPO, a) if a.endswith(".py") else a for a in argv]


@pytest.mark.parametrize("argv,case", CASES)
def test_custom_roots_resolve(argv, case):
    """--custom/--init_pos take effect (the reference silently ignores them)."""
    args = solver_launcher.build_parser().parse_args(_abs(argv))
    game, root = solver_launcher.prepare_game(args)
    assert str(root) == ROOTS[case]["root"]


def test_missing_custom_file_falls_back(capsys):
    args = solver_launcher.build_parser().parse_args(
        _abs(["test_games/mttt.py", "--init_pos", "x"]) + ["--custom", "/nonexistent.py"])
    game, root = solver_launcher.prepare_game(args)
    assert root == "_" * 9
    assert "Custom file was not found" in capsys.readouterr().out


def test_validate_rejects_incomplete_plugin(tmp_path):
    bad = tmp_path / "bad.py"
    bad.write_text("def initial_position():\n    return 1\n")
    args = solver_launcher.build_parser().parse_args([str(bad)])
    with pytest.raises(AttributeError):
        solver_launcher.prepare_game(args)


def test_dims_flag_patches_board_plugins():
    args = solver_launcher.build_parser().parse_args(
        _abs(["test_games/toot_and_otto_bitstring.py"]) + ["--dims", "4x3"])
    game, root = solver_launcher.prepare_game(args)
    assert (game.length, game.height) == (4, 3) and len(root) == 6


def test_rank_plan():
    """mpiexec -n N semantics (reference solver_launcher.py:43-60): one GPU per rank ->
    sharded; more ranks than GPUs (the reference's --oversubscribe tests) -> rank 0
    solves for all."""
    plan = solver_launcher.rank_plan
    assert plan(1, 1, 0) == "solo" and plan(1, 1, 8) == "solo"
    assert plan(2, 2, 8) == "sharded" and plan(8, 8, 8) == "sharded"
    assert plan(5, 5, 1) == "single" and plan(2, 2, 1) == "single" and plan(9, 9, 8) == "single"
    assert plan(4, 2, 8) == "single"   # two nodes: the RCCL solve is single-node


_SINGLE_MODE_RANK = r'''
import io, json, os, sys
sys.path.insert(0, sys.argv[1])
os.environ.update(RANK=sys.argv[2], LOCAL_RANK=sys.argv[2], WORLD_SIZE=sys.argv[3], LOCAL_WORLD_SIZE=sys.argv[3],
                  MASTER_ADDR="127.0.0.1", MASTER_PORT=sys.argv[4])
import solver_launcher, gamesmanmpi_amd
seen = {}
class FakeCtx:
    def set_option(self, opt, v): seen[opt] = v
    def stats(self): return {}
class FakeSolver:   # stands in for the GPU solve (this container has no GPU)
    def __init__(self, module, root, device=-1, engine=None):
        from gamesmanmpi_amd import games
        self.codec, self.ctx = games.FourToOneCodec(), FakeCtx()
        seen["device"] = device
    def solve(self):
        import time
        time.sleep(float(os.environ.get("FAKE_SOLVE_S", "0")))
    def root_line(self): return "WIN in 3 moves"
    def close(self): pass
gamesmanmpi_amd.Solver = FakeSolver
out = io.StringIO()
args = solver_launcher.build_parser().parse_args([os.path.join(sys.argv[1], "test_games/four_to_one.py")])
rc = solver_launcher.run(args, out=out)
print(json.dumps({"rc": rc, "out": out.getvalue(), "seen": {str(k): v for k, v in seen.items()}}))
'''


@pytest.mark.parametrize("solve_s,timeout_s", [(0, None), (6, 2)])
def test_launcher_single_mode_ranks_gloo(tmp_path, solve_s, timeout_s):
    """More launcher ranks than GPUs (this container has none): rank 0 solves with
    world loopback ranks (GM_OPT_VIRTUAL_RANKS) and prints the one root line; the
    other ranks print nothing, wait for rank 0 and return 0 -- also when rank 0's solve
    (6 s) outlasts the gloo group's timeout (2 s, GM_DIST_TIMEOUT_S): they poll the
    group's store instead of waiting in a collective."""
    import socket
    import subprocess
    import sys
    from gamesmanmpi_amd import _lib
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    world = 3
    env = dict(os.environ, FAKE_SOLVE_S=str(solve_s))
    if timeout_s is not None:
        env["GM_DIST_TIMEOUT_S"] = str(timeout_s)
    procs = [subprocess.Popen([sys.executable, "-c", _SINGLE_MODE_RANK, REPO, str(r), str(world), str(port)],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
             for r in range(world)]
    res = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=120)
            assert p.returncode == 0, e
            res.append(json.loads(o.strip().splitlines()[-1]))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert all(r["rc"] == 0 for r in res)
    assert res[0]["out"] == "WIN in 3 moves\n" and all(r["out"] == "" for r in res[1:])
    assert res[0]["seen"] == {str(_lib.OPT_VIRTUAL_RANKS): world, "device": -1}
    assert all(r["seen"] == {} for r in res[1:])


@pytest.mark.gpu
@pytest.mark.parametrize("argv,case", CASES)
def test_launcher_root_lines(argv, case):
    out = io.StringIO()
    args = solver_launcher.build_parser().parse_args(_abs(argv))
    assert solver_launcher.run(args, out=out) == 0
    assert out.getvalue() == ROOTS[case]["canonical"] + "\n"


def _torchrun(nproc, argv, timeout=180):
    import socket
    import subprocess
    import sys
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(REPO, "solver_launcher.py")] + _abs(argv)
    return subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=timeout,
                          env=dict(os.environ, PYTHONUNBUFFERED="1"))


@pytest.mark.gpu
@pytest.mark.parametrize("argv,case", CASES)
def test_launcher_under_torchrun_more_ranks_than_gpus(argv, case):
    """The reference's game_tests run the launcher as `mpiexec --oversubscribe -n 2`
    (four_to_one_test.py:14-23); BASELINE config 1 is `-n 5`.  Here: torch.distributed.run
    with 5 ranks (Four-To-One) or 2 (mttt) on a one-GPU box; stdout must be exactly the
    one root line."""
    nproc = 5 if case.startswith("four_to_one") else 2
    r = _torchrun(nproc, argv)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout == ROOTS[case]["canonical"] + "\n", (r.stdout, r.stderr[-2000:])


@pytest.mark.gpu
def test_launcher_statsdir_dump(tmp_path):
    import numpy as np
    args = solver_launcher.build_parser().parse_args(_abs(["test_games/mttt.py"]) + ["-sd", str(tmp_path)])
    solver_launcher.run(args, out=io.StringIO())
    d = np.load(tmp_path / "stats" / "0" / "table.npz")
    g = np.load(os.path.join(GOLDEN, "ttt.npz"))
    assert (d["keys"] == g["keys"]).all() and (d["records"] == g["records"]).all()
    # the reference's shelve layout (src/cache_dict.py:19-42), keyed by the mttt boards
    from gamesmanmpi_amd import games
    from gamesmanmpi_amd.persist import read_reference_tables
    back = read_reference_tables(str(tmp_path))
    codec = games.TTTStringCodec()
    assert len(back) == 5478
    for k, r in zip(g["keys"].tolist(), g["records"].tolist()):
        assert back[codec.pos(k)] == (r >> 14, r & 0x3FFF)


@pytest.mark.gpu
def test_solve_local_messages(capsys):
    solve_local.main([os.path.join(REPO, "test_games/four_to_one.py")])
    solve_local.main([os.path.join(REPO, "test_games/mttt.py"), "--remoteness"])
    solve_local.main([os.path.join(REPO, "test_games/othello_bit_new.py"), "--dims", "4x4"])
    assert capsys.readouterr().out.splitlines() == [
        "Winning position", "Tie", "TIE in 9 moves", "Losing position"]


@pytest.mark.gpu
def test_launcher_othello_8x8_endgame_on_the_device(tmp_path):
    """`solver_launcher.py tests/plugins/othello8_endgame.py -sd DIR`: the 8x8 plugin binds the
    128-bit-key descriptor, the launcher prints the canonical root line, and -sd writes the
    (n, 3)-word key table and the reference's shelves, every record equal to the reference
    plugin's golden table (keys = blake2b-8 of the position string)."""
    import hashlib
    import json
    import numpy as np
    from gamesmanmpi_amd.persist import read_reference_tables
    args = solver_launcher.build_parser().parse_args(_abs(["tests/plugins/othello8_endgame.py"])
                                                     + ["-sd", str(tmp_path), "--sd-format", "both"])
    out = io.StringIO()
    solver_launcher.run(args, out=out)
    roots = json.load(open(os.path.join(GOLDEN, "roots.json")))
    assert out.getvalue() == roots["othello_8x8_endgame"]["canonical"] + "\n"
    d = np.load(tmp_path / "stats" / "0" / "table.npz")
    assert d["keys"].shape == (56552, 3)
    back = read_reference_tables(str(tmp_path))
    g = np.load(os.path.join(GOLDEN, "othello_8x8_endgame.npz"))
    want = dict(zip(g["keys"].tolist(), g["records"].tolist()))
    got = {int.from_bytes(hashlib.blake2b(p.encode("ISO-8859-1"), digest_size=8).digest(), "big"): (v << 14) | r
           for p, (v, r) in back.items()}
    assert got == want


@pytest.mark.gpu
def test_launcher_othello_8x8_custom_root_on_the_device(tmp_path, capsys):
    """`solver_launcher.py test_games/othello_bit_new.py --custom tools/othello8_roots.py
    --init_pos endgame_10`: the unmodified plugin with the root from a custom file (the
    reference's launcher patches initial_position, solver_launcher.py:106-111) keeps the
    device binding -- the hash-sharded sparse engine, not the graph path -- and every record
    equals the reference plugin's golden table for that root."""
    import hashlib
    import json
    import numpy as np
    from gamesmanmpi_amd import _lib
    args = solver_launcher.build_parser().parse_args(
        _abs(["test_games/othello_bit_new.py", "--custom", "tools/othello8_roots.py"])
        + ["--init_pos", "endgame_10", "--stats", "-sd", str(tmp_path), "--sd-format", "npz"])
    out = io.StringIO()
    solver_launcher.run(args, out=out)
    roots = json.load(open(os.path.join(GOLDEN, "roots.json")))
    assert out.getvalue() == roots["othello_8x8_endgame"]["canonical"] + "\n"
    stats = json.loads(capsys.readouterr().err.strip().splitlines()[-1])
    assert stats["engine"] == _lib.ENGINE_DIST_SPARSE
    d = np.load(tmp_path / "stats" / "0" / "table.npz")
    g = np.load(os.path.join(GOLDEN, "othello_8x8_endgame.npz"))
    want = dict(zip(g["keys"].tolist(), g["records"].tolist()))
    got = {}
    for w, r in zip(d["keys"].tolist(), d["records"].tolist()):
        pos = sum(int(x) << (64 * i) for i, x in enumerate(w)).to_bytes(18, "big")
        got[int.from_bytes(hashlib.blake2b(pos, digest_size=8).digest(), "big")] = int(r)
    assert got == want
