"""Tic-tac-toe where a full board without a line is a LOSS for the player to move
(instead of the reference mttt's TIE), in the reference's 9-char string encoding.
No descriptor reproduces it, so it goes through the explicit-graph engine."""
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
    return UNDECIDED if "_" in pos else LOSS
