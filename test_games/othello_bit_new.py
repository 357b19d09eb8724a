"""Othello on a ``length`` x ``height`` bitboard, positions packed into latin-1 strings.

Same position encoding and rules as the reference ``test_games/othello_bit_new.py``
(built there with the third-party ``bitstring.BitArray``; here a Python int):

* bits MSB-first; ``[0, A)`` WHITE plane and ``[A, 2A)`` BLACK plane, cell ``(x, y)``
  at ``length*y + x`` (``:241-271``);
* an 8-bit signed turn count (1 = BLACK to move, 2 = WHITE) at ``2A`` and an 8-bit
  pass count at ``2A + 8`` (``:14``, ``:278-306``), padded to whole bytes;
* the start has WHITE on the two diagonal centre cells and the turn advanced
  twice from 0, so WHITE moves first (``:36-55``);
* moves are scanned x outer, y inner; a cell is legal when some direction holds a
  run of opponent pieces closed by an own piece; with no legal cell the only move
  is ``None`` (``:132-170``);
* ``None`` increments the pass count and does NOT hand the turn over; a placement
  resets the pass count, flips bracketed runs in all 8 directions and hands the
  turn over (``:86-130``; flip bounds test ``x`` against ``height`` as the reference
  does, which only matters on non-square boards);
* the game ends on a full board or two passes; the side to move wins with more
  pieces (``:57-84``).

Default dimensions are the reference's 8x8; the solver configs patch 4x4.
"""
import src.utils as U

length, height = 8, 8
BLANK, WHITE, BLACK = 0, 2, 1
opponent = {BLACK: WHITE, WHITE: BLACK, BLANK: BLANK}
char_rep = {BLACK: "O", WHITE: "X", BLANK: "-"}
turn_count_map = {1: BLACK, 2: WHITE}
_DIRS = tuple((dx, dy) for dx in (-1, 0, 1) for dy in (-1, 0, 1) if dx or dy)


def _geom():
    a = length * height
    nbits = -(-(2 * a + 16) // 8) * 8
    return a, nbits


def _load(pos):
    return int.from_bytes(pos.encode("ISO-8859-1"), "big")


def _store(v, nbits):
    return v.to_bytes(nbits // 8, "big").decode("ISO-8859-1")


def _get(v, j, nbits):
    return (v >> (nbits - 1 - j)) & 1


def _put(v, j, nbits, bit):
    mask = 1 << (nbits - 1 - j)
    return (v | mask) if bit else (v & ~mask)


def _cell(v, x, y, a, nbits):
    if _get(v, int(length * y + x), nbits):
        return WHITE
    if _get(v, int(a + length * y + x), nbits):
        return BLACK
    return BLANK


def _paint(v, x, y, color, a, nbits):
    w, b = int(length * y + x), int(a + length * y + x)
    v = _put(v, w, nbits, color == WHITE)
    return _put(v, b, nbits, color == BLACK)


def _field(v, start, nbits):
    raw = (v >> (nbits - start - 8)) & 0xFF
    return raw - 256 if raw >= 128 else raw


def _set_field(v, start, nbits, value):
    shift = nbits - start - 8
    return (v & ~(0xFF << shift)) | ((value & 0xFF) << shift)


def _turn(v, a, nbits):
    return _field(v, 2 * a, nbits)


def _mover(v, a, nbits):
    return turn_count_map[_turn(v, a, nbits)]


def initial_position():
    a, nbits = _geom()
    v = 0
    v = _paint(v, length / 2 - 1, height / 2 - 1, WHITE, a, nbits)
    v = _paint(v, length / 2 - 1, height / 2, BLACK, a, nbits)
    v = _paint(v, length / 2, height / 2 - 1, BLACK, a, nbits)
    v = _paint(v, length / 2, height / 2, WHITE, a, nbits)
    for _ in range(2):
        v = _set_field(v, 2 * a, nbits, _turn(v, a, nbits) % 2 + 1)
    return _store(v, nbits)


def primitive(pos):
    a, nbits = _geom()
    v = _load(pos)
    cells = [_cell(v, x, y, a, nbits) for x in range(length) for y in range(height)]
    filled = sum(1 for c in cells if c != BLANK)
    if filled != a and _field(v, 2 * a + 8, nbits) < 2:
        return U.UNDECIDED
    black = cells.count(BLACK)
    white = cells.count(WHITE)
    if black == white:
        return U.TIE
    if (black > white) ^ (_turn(v, a, nbits) == 1):
        return U.LOSS
    return U.WIN


def _brackets(v, x, y, dx, dy, me, a, nbits):
    them = opponent[me]
    x, y = x + dx, y + dy
    seen = 0
    while 0 <= x < length and 0 <= y < height:
        c = _cell(v, x, y, a, nbits)
        if c == them:
            seen += 1
        elif c == me:
            return seen > 0
        else:
            return False
        x, y = x + dx, y + dy
    return False


def gen_moves(pos):
    a, nbits = _geom()
    v = _load(pos)
    me = _mover(v, a, nbits)
    out = []
    for x in range(length):
        for y in range(height):
            if _cell(v, x, y, a, nbits) != BLANK:
                continue
            if any(_brackets(v, x, y, dx, dy, me, a, nbits) for dx, dy in _DIRS):
                out.append((x, y))
    return out or [None]


def do_move(pos, move):
    a, nbits = _geom()
    v = _load(pos)
    if move is None:
        return _store(_set_field(v, 2 * a + 8, nbits, _field(v, 2 * a + 8, nbits) + 1), nbits)
    v = _set_field(v, 2 * a + 8, nbits, 0)
    me = _mover(v, a, nbits)
    them = opponent[me]
    x, y = move
    v = _paint(v, x, y, me, a, nbits)
    for dx, dy in _DIRS:
        run = []
        cx, cy = x + dx, y + dy
        while not (cx >= height or cy >= length or cx < 0 or cy < 0):
            c = _cell(v, cx, cy, a, nbits)
            if c == them:
                run.append((cx, cy))
            elif c == me:
                for fx, fy in run:
                    v = _paint(v, fx, fy, me, a, nbits)
                break
            else:
                break
            cx, cy = cx + dx, cy + dy
    v = _set_field(v, 2 * a, nbits, _turn(v, a, nbits) % 2 + 1)
    return _store(v, nbits)


def symmetry_functions():
    """Declared by the reference (``:224-225``) and never called by its solver."""
    return []
