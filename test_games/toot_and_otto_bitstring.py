"""Toot-and-Otto on a ``length`` x ``height`` board, positions packed into latin-1 strings.

Same position encoding and rules as the reference
``test_games/toot_and_otto_bitstring.py`` (which builds them with the third-party
``bitstring.BitArray``; here the same bits are handled as a Python int):

* bits are numbered MSB-first over the whole string;
* ``[0, A)``: T plane, cell ``(x, y)`` at ``length*y + x`` (A = length*height, ``:179-199``);
* ``[A, 2A)``: O plane, same indexing;
* then four signed 4-bit hand counts: player-1 T, player-1 O, player-2 T, player-2 O,
  each starting at 6 (``:39-40``, ``:202-216``);
* one constant 1 bit, then zero padding to a whole byte (``:41-43``);
* the LAST padding bit is the turn bit: set means player 1 to move (``:218-222``).
  It starts clear, so player 2 moves first.

Moves are ``(x, T)`` / ``(x, O)`` for every column whose top cell is empty, if the
mover still holds that letter (``:87-100``); the letter drops to the lowest empty
cell (``:102-115``).  TOOT/OTTO occurrences are counted from every piece in the
directions (1,0), (0,1), (1,1), (1,-1) (``:46-85``).

``length``/``height`` are read at call time, so tests may patch them.
"""
import src.utils as U

length, height = 6, 4
BLANK, T, O = 0, 1, -1
char_rep = {T: "T", O: "O", BLANK: "-"}
TOOT, OTTO = "TOOT", "OTTO"
_DIRS = ((1, 0), (0, 1), (1, 1), (1, -1))


def _geom():
    a = length * height
    nbits = -(-(2 * a + 17) // 8) * 8
    return a, nbits


def _load(pos):
    return int.from_bytes(pos.encode("ISO-8859-1"), "big")


def _store(v, nbits):
    return v.to_bytes(nbits // 8, "big").decode("ISO-8859-1")


def _get(v, j, nbits):
    return (v >> (nbits - 1 - j)) & 1


def _set(v, j, nbits, bit):
    mask = 1 << (nbits - 1 - j)
    return (v | mask) if bit else (v & ~mask)


def _cell(v, x, y, a, nbits):
    if _get(v, length * y + x, nbits):
        return T
    if _get(v, a + length * y + x, nbits):
        return O
    return BLANK


def _hand_slot(a, player, letter):
    return 2 * a + 8 * (player - 1) + (0 if letter == T else 4)


def _hand(v, player, letter, a, nbits):
    start = _hand_slot(a, player, letter)
    raw = (v >> (nbits - start - 4)) & 0xF
    return raw - 16 if raw >= 8 else raw


def _player1_to_move(v):
    return bool(v & 1)


def initial_position():
    a, nbits = _geom()
    v = 0
    for k in range(4):
        v |= 0b0110 << (nbits - (2 * a + 4 * k) - 4)
    v = _set(v, 2 * a + 16, nbits, 1)
    return _store(v, nbits)


def _score(v, a, nbits):
    found = {TOOT: 0, OTTO: 0}
    for x in range(length):
        for y in range(height):
            c = _cell(v, x, y, a, nbits)
            if c == BLANK:
                continue
            word = TOOT if c == T else OTTO
            for dx, dy in _DIRS:
                ok = True
                for k in range(1, 4):
                    xx, yy = x + k * dx, y + k * dy
                    if not (0 <= xx < length and 0 <= yy < height) or \
                            char_rep[_cell(v, xx, yy, a, nbits)] != word[k]:
                        ok = False
                        break
                if ok:
                    found[word] += 1
    return found


def _full(v, a, nbits):
    return all(_cell(v, x, y, a, nbits) != BLANK
               for x in range(length) for y in range(height))


def primitive(pos):
    a, nbits = _geom()
    v = _load(pos)
    s = _score(v, a, nbits)
    if s[TOOT] == s[OTTO]:
        return U.TIE if _full(v, a, nbits) else U.UNDECIDED
    if (s[TOOT] > s[OTTO]) ^ _player1_to_move(v):
        return U.LOSS
    return U.WIN


def gen_moves(pos):
    a, nbits = _geom()
    v = _load(pos)
    player = 1 if _player1_to_move(v) else 2
    have_t = _hand(v, player, T, a, nbits) > 0
    have_o = _hand(v, player, O, a, nbits) > 0
    out = []
    for x in range(length):
        if _cell(v, x, height - 1, a, nbits) == BLANK:
            if have_t:
                out.append((x, T))
            if have_o:
                out.append((x, O))
    return out


def do_move(pos, move):
    a, nbits = _geom()
    v = _load(pos)
    x, letter = move
    player = 1 if _player1_to_move(v) else 2
    start = _hand_slot(a, player, letter)
    count = (_hand(v, player, letter, a, nbits) - 1) & 0xF
    shift = nbits - start - 4
    v = (v & ~(0xF << shift)) | (count << shift)
    v ^= 1  # toggle the turn bit (the last bit)
    for y in range(height):
        if _cell(v, x, y, a, nbits) == BLANK:
            t_bit, o_bit = length * y + x, a + length * y + x
            v = _set(v, t_bit, nbits, letter == T)
            v = _set(v, o_bit, nbits, letter == O)
            return _store(v, nbits)
    return None  # column full: the reference also returns None here (:112-115)
