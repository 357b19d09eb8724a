"""Four-To-One: a pile of 4; a move removes 1 or 2; facing a pile <= 0 is a loss.

Same plugin contract and position encoding as the reference
``test_games/four_to_one.py:8-31``: positions are decimal strings (the shelve-key
convention of ``src.utils.encode_int``).

Quirk kept for parity: the reference's ``gen_moves`` receives the position as a
string, so its ``x == 1`` test (``four_to_one.py:15``) never fires and the moves
are always ``-1, -2``.  A pile of 1 therefore has the children 0 and -1.
"""
import src.utils as U


@U.encode_int
def initial_position():
    return 4


def gen_moves(pos):
    return ["-1", "-2"]


@U.decode_int
@U.encode_int
def do_move(pos, move):
    return pos + move


@U.decode_int
def primitive(pos):
    return U.LOSS if pos <= 0 else U.UNDECIDED
