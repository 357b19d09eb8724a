"""Tic-tac-toe on a 9-character string of 'X', 'O' and '_'.

Same encoding and rules as the reference ``test_games/mttt.py:11-127``:
cell ``(x, y)`` is character ``x + 3*y``; X is to move whenever O has at least as
many pieces; three equal pieces in a row, column or diagonal make the position
a LOSS for the player to move; a full board without such a line is a TIE.
"""
import src.utils as U

WIDTH = 3
HEIGHT = 3
X, O, BLANK = "X", "O", "_"
BORDER = "B"

_LINES = ((0, 1, 2), (3, 4, 5), (6, 7, 8),
          (0, 3, 6), (1, 4, 7), (2, 5, 8),
          (0, 4, 8), (2, 4, 6))


def initial_position():
    return BLANK * (WIDTH * HEIGHT)


def to_loc(i):
    return i % WIDTH, i // WIDTH


def to_index(loc):
    return loc[0] + WIDTH * loc[1]


def get_player(pos):
    return X if pos.count(O) >= pos.count(X) else O


def primitive(pos):
    for a, b, c in _LINES:
        if pos[a] != BLANK and pos[a] == pos[b] == pos[c]:
            return U.LOSS
    return U.UNDECIDED if BLANK in pos else U.TIE


def gen_moves(pos):
    return [to_loc(i) for i, ch in enumerate(pos) if ch == BLANK]


def do_move(pos, move):
    i = to_index(move)
    return pos[:i] + get_player(pos) + pos[i + 1:]
