"""Custom roots for mttt (the boards of the reference's game_tests/mttt_test_init_pos.py).

Like the reference file, it reads the piece symbols from the loaded plugin.
"""
import src.utils

_g = src.utils.game_module
X, O, B = _g.X, _g.O, _g.BLANK


def tie_in_one():
    return "".join([X, X, O, O, O, X, X, O, B])


def win_in_one():
    return "".join([X, X, B, O, O, X, X, O, O])


def side_columns():
    return "".join([X, B, O, O, B, X, X, B, O])


def one_row():
    return "".join([X, X, O, B, B, B, B, B, B])
