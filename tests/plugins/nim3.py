"""Three-heap subtraction game in the reference's plugin style (no device descriptor).

Positions are (a, b, c) tuples; a move removes 1..3 from one heap; no heap left
means the player to move has lost.  Used to test the explicit-graph engine on a
plugin that games.identify() cannot match.
"""
from src.utils import LOSS, UNDECIDED

START = (5, 6, 7)


def initial_position():
    return START


def gen_moves(pos):
    return [(i, t) for i in range(3) for t in (1, 2, 3) if pos[i] >= t]


def do_move(pos, move):
    i, t = move
    out = list(pos)
    out[i] -= t
    return tuple(out)


def primitive(pos):
    return LOSS if not any(pos) else UNDECIDED
