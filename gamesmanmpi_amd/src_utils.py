"""Result-code names used by the host (mirrors reference src/utils.py:4, :61-67)."""

_NAMES = ("WIN", "LOSS", "TIE", "DRAW", "UNDECIDED")


def to_str(state):
    return _NAMES[state]
