"""Custom roots for Four-To-One (the positions of the reference's game_tests/four_to_one_init_pos.py)."""
import src.utils as U


@U.encode_int
def six():
    return 6


@U.encode_int
def one():
    return 1


@U.encode_int
def zero():
    return 0
