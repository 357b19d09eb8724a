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


@pytest.mark.gpu
@pytest.mark.parametrize("argv,case", CASES)
def test_launcher_root_lines(argv, case):
    out = io.StringIO()
    args = solver_launcher.build_parser().parse_args(_abs(argv))
    assert solver_launcher.run(args, out=out) == 0
    assert out.getvalue() == ROOTS[case]["canonical"] + "\n"


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
