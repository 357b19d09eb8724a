"""Tic-tac-toe that differs from the reference mttt (test_games/mttt.py) only on boards
with at least 7 pieces: there a completed line is a WIN for the player to move
instead of a LOSS.  Every position with up to 6 pieces -- the whole BFS prefix and
most of any random playout -- behaves exactly like mttt, so only an exhaustive
check can tell the two apart; games.identify must not bind it to the TTT descriptor."""
from src.utils import LOSS, TIE, UNDECIDED, WIN

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
            return WIN if 9 - pos.count("_") >= 7 else LOSS
    return UNDECIDED if "_" in pos else TIE
