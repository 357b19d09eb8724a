"""Tic-tac-toe on a 3x3 ``np.int8`` board (0 empty, 1 and 2 the players).

Same encoding and rules as the reference ``test_games/tic_tac_toe_np.py:7-61``:
player 1 moves unless it already has more pieces than player 2; a move is
``(player, (x, y))`` and sets ``state[x][y]``; any three equal non-empty cells in
a line make the position a LOSS for the player to move; a full board is a TIE.
(The reference also imports mpi4py without using it; that import is dropped.)
"""
import numpy as np

import src.utils as U

_LINES = tuple(
    tuple((x, y) for x, y in line) for line in (
        [(0, 0), (1, 0), (2, 0)], [(0, 1), (1, 1), (2, 1)], [(0, 2), (1, 2), (2, 2)],
        [(0, 0), (0, 1), (0, 2)], [(1, 0), (1, 1), (1, 2)], [(2, 0), (2, 1), (2, 2)],
        [(0, 0), (1, 1), (2, 2)], [(0, 2), (1, 1), (2, 0)]))


def initial_position():
    return np.zeros((3, 3), dtype=np.int8)


def _mover(state):
    ones = int(np.count_nonzero(state == 1))
    twos = int(np.count_nonzero(state == 2))
    return 2 if ones > twos else 1


def gen_moves(state):
    who = _mover(state)
    return [(who, (x, y)) for x in range(3) for y in range(3) if state[x][y] == 0]


def do_move(state, action):
    child = state.copy()
    who, (x, y) = action
    child[x, y] = who
    return child


def primitive(state):
    for (a, b, c) in _LINES:
        v = state[a]
        if v != 0 and state[b] == v and state[c] == v:
            return U.LOSS
    return U.TIE if np.count_nonzero(state) == 9 else U.UNDECIDED
