"""Endgame roots for the reference's 8x8 Othello plugin, as a ``--custom`` file of the launcher:

    python solver_launcher.py test_games/othello_bit_new.py --custom tools/othello8_roots.py --init_pos endgame_16

Positions of the seed-5 playout from the standard start with E empty squares (bench.py
OTHELLO8_ROOTS; tools/othello8_scale.py playout_roots).  The plugin keeps its code, so the
launcher binds the device descriptor by its fingerprint.
"""


def _pos(h):
    return bytes.fromhex(h).decode("latin-1")


def endgame_10():
    return _pos("303800204018057a4646bfdebfe6fa800200")


def endgame_14():
    return _pos("30300c2c503841784646b1d2afc6be000200")


def endgame_16():
    return _pos("3030242050384178460699daafc6be000200")
