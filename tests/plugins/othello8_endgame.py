"""Othello on the reference's default 8x8 board, solved from an endgame position.

The plugin functions are test_games/othello_bit_new.py's (8x8, as the reference ships it,
`othello_bit_new.py:8`); only the root differs: the position after a fixed random playout
from the standard start (seed 5), 10 empty squares left, 56,552 positions below it.  An 8x8
position is 2A + 16 = 144 bits; the rules are the plugin's own code, so the solver binds the
128-bit-key descriptor by their fingerprint (`graph=True` takes the
explicit-graph path instead, tests/test_graph.py).  The golden table
(tests/golden/othello_8x8_endgame.npz) is the canonical solution of the REFERENCE's plugin
from the same root (tests/golden/make_golden.py --only othello8).
"""
import os

from test_games.othello_bit_new import *  # noqa: F401,F403  (the game: moves, rules, encoding)
from test_games.othello_bit_new import do_move, gen_moves, primitive  # noqa: F401

# GM_OTHELLO8_ROOT (a position string in hex) replaces the root for scale runs: the same
# playout stopped earlier, 12 empties "30380028503841784646bfd6afc6be000200", 13
# "30381c2c503841784646a1d2afc6be000100" 
ROOT_HEX = os.environ.get("GM_OTHELLO8_ROOT", "303800204018057a4646bfdebfe6fa800200")


def initial_position():
    return bytes.fromhex(ROOT_HEX).decode("latin-1")
