"""Plugin-facing constants and helpers (drop-in for the reference's ``src.utils``).

Game plugins written for GamesmanMPI do ``import src.utils`` and read the result
codes and the ``encode_int``/``decode_int`` decorators from it
(reference ``test_games/four_to_one.py:5``, ``src/utils.py:4-46``).  This module
provides the same names with the same numeric values so unmodified plugin files
import against this tree.  Nothing here is on the solve path: the solver reads
results from the GPU library (``gamesmanmpi_amd``).
"""

# Result codes, from the perspective of the player to move (reference src/utils.py:4).
WIN, LOSS, TIE, DRAW, UNDECIDED = 0, 1, 2, 3, 4
PRIMITIVES = (WIN, LOSS, TIE, DRAW)
DWULT = PRIMITIVES
PRIMITIVE_REMOTENESS = 0          # src/utils.py:7
UNKNOWN_REMOTENESS = -1           # src/utils.py:8

# The loaded plugin; set by solver_launcher.py / solve_local.py (src/utils.py:9).
game_module = None

_NAMES = ("WIN", "LOSS", "TIE", "DRAW", "UNDECIDED")
STATE_MAP = {code: name.lower() for code, name in enumerate(_NAMES)}


def to_str(state):
    """``to_str(LOSS) == 'LOSS'`` (src/utils.py:61-67)."""
    return _NAMES[state]


def negate(state):
    """WIN <-> LOSS; every other code is its own negation (src/utils.py:49-58)."""
    if state == WIN:
        return LOSS
    if state == LOSS:
        return WIN
    return state


def encode_int(f):
    """Decorator: int results become str (a list result becomes a list of str).

    The reference stores positions as shelve keys, so integer plugins return
    strings (src/utils.py:22-34).  The reference returns a lazy ``map`` for
    lists; a list is returned here so callers may iterate it more than once.
    """
    def wrapped(*args):
        out = f(*args)
        if isinstance(out, list):
            return [str(v) for v in out]
        return str(out)
    wrapped.__name__ = getattr(f, "__name__", "encoded")
    wrapped.__doc__ = f.__doc__
    return wrapped


def decode_int(f):
    """Decorator: every positional argument is passed through ``int`` (src/utils.py:37-46)."""
    def wrapped(*args):
        return f(*(int(a) for a in args))
    wrapped.__name__ = getattr(f, "__name__", "decoded")
    wrapped.__doc__ = f.__doc__
    return wrapped


def reduce_singleton(function, data):
    """``reduce`` that also accepts a single element (src/utils.py:70-77)."""
    items = list(data)
    if len(items) == 1:
        return function(items[0], None)
    acc = items[0]
    for item in items[1:]:
        acc = function(acc, item)
    return acc


def get_hash(pos, world_size):
    """Owner rank of a position: md5 of ``str(pos)`` mod world size (src/utils.py:80-87).

    Kept for API compatibility; the GPU solver uses its own owner function.
    """
    import hashlib
    digest = hashlib.md5(str(pos).encode("utf-8")).hexdigest()
    return int(digest, 16) % world_size


def argmin(a, b, index):
    """Tuple with the smaller ``[index]``; ``a`` on ties (src/utils.py:90-96)."""
    return a if a[index] <= b[index] else b


def argmax(a, b, index):
    """Tuple with the larger ``[index]``; ``a`` on ties (src/utils.py:99-105)."""
    return a if a[index] >= b[index] else b
