"""Generalised subtraction game: the synthetic 2^32-state config.

Not part of the reference; it generalises Four-To-One (``test_games/four_to_one.py``)
to ``HEAPS`` heaps of 0..15 tokens packed 4 bits per heap into one int
(heap ``i`` in bits ``[4i, 4i+4)``).  A move removes 1 or 2 tokens from one
non-empty heap, never going below 0 (so a heap of 1 has one move, not two);
facing all heaps empty is a LOSS.  With ``HEAPS = 1`` the values and remoteness
equal Four-To-One's for piles >= 0.

``HEAPS`` is read at call time, so tests may patch it.
"""
import src.utils as U

HEAPS = 8
BITS = 4
MAX_TAKE = 2


def initial_position():
    return (1 << (BITS * HEAPS)) - 1


def _heap(pos, i):
    return (pos >> (BITS * i)) & ((1 << BITS) - 1)


def gen_moves(pos):
    moves = []
    for i in range(HEAPS):
        h = _heap(pos, i)
        for take in range(1, MAX_TAKE + 1):
            if h >= take or (take == 1 and h >= 1):
                moves.append((i, take))
    return moves


def do_move(pos, move):
    i, take = move
    h = _heap(pos, i)
    return pos - (min(h, take) << (BITS * i))


def primitive(pos):
    return U.LOSS if pos == 0 else U.UNDECIDED
