"""Tic-tac-toe (the reference mttt's rules and 9-char board) that declares the square's
symmetries through the reference's hook ``symmetry_functions()`` -- a list of
``(function, order)`` pairs, as othello_bit_new.py:224-225 declares player_flip.  The
graph engine uses the declared functions that fix the root: from the empty board all
eight board symmetries, so 5,478 positions are solved as 765 orbits."""
from src.utils import LOSS, TIE, UNDECIDED

LINES = [(0, 1, 2), (3, 4, 5), (6, 7, 8), (0, 3, 6), (1, 4, 7), (2, 5, 8), (0, 4, 8), (2, 4, 6)]


def initial_position():
    return "_" * 9


def gen_moves(pos):
    return [i for i, ch in enumerate(pos) if ch == "_"]


def do_move(pos, i):
    mover = "X" if pos.count("O") >= pos.count("X") else "O"
    return pos[:i] + mover + pos[i + 1:]


def primitive(pos):
    for a, b, c in LINES:
        if pos[a] != "_" and pos[a] == pos[b] == pos[c]:
            return LOSS
    return UNDECIDED if "_" in pos else TIE


def rotate(pos):      # (x, y) -> (2 - y, x), cell i = x + 3y
    return "".join(pos[(2 - (i % 3)) * 3 + (i // 3)] for i in range(9))


def mirror(pos):      # (x, y) -> (2 - x, y)
    return "".join(pos[3 * (i // 3) + 2 - (i % 3)] for i in range(9))


def symmetry_functions():
    return [(rotate, 4), (mirror, 2)]
