"""Plugin positions <-> descriptor keys, and plugin -> descriptor matching.

A GamesmanMPI plugin (``initial_position / gen_moves / do_move / primitive``,
reference README.md:28-88) is solved on the GPU when one of the device
descriptors (gamesmanmpi_amd/csrc/games.hpp) reproduces it.  ``identify()``
finds that descriptor: each codec below converts the plugin's positions to u64
keys, and a match must be certain: a known plugin file
(code fingerprint, gamesmanmpi_amd/fingerprint.py) or an exhaustive replay of the
plugin against the descriptor's host twin (``gm_expand_host``) -- primitive values
and child sets must agree exactly on every reachable position.
"""
import os
import random

import numpy as np

from . import _lib

MASK64 = (1 << 64) - 1
_DIGIT = {"_": 0, "X": 1, "O": 2}
_CHAR = "_XO"


class Codec:
    game_id = 0
    params = ()
    name = "?"

    def key(self, pos):
        raise NotImplementedError

    def pos(self, key):
        raise NotImplementedError


class FourToOneCodec(Codec):
    """Decimal-string piles (reference test_games/four_to_one.py, src/utils.py:22-46)."""
    game_id = _lib.GAME_FOUR_TO_ONE
    name = "four_to_one"

    def key(self, pos):
        if isinstance(pos, (bool, np.ndarray)):
            raise ValueError("not a Four-To-One position")
        x = int(pos)
        if not -(1 << 60) < x < (1 << 60):
            raise ValueError("pile out of range")
        return x & MASK64

    def pos(self, key):
        x = key - (1 << 64) if key >> 63 else key
        return str(x)


class TTTStringCodec(Codec):
    """9-char 'X'/'O'/'_' boards (reference test_games/mttt.py)."""
    game_id = _lib.GAME_TTT
    name = "mttt"

    def key(self, pos):
        if not isinstance(pos, str) or len(pos) != 9 or any(c not in _DIGIT for c in pos):
            raise ValueError("not a mttt board")
        return sum(_DIGIT[c] * 3 ** i for i, c in enumerate(pos))

    def pos(self, key):
        out = []
        for _ in range(9):
            out.append(_CHAR[key % 3])
            key //= 3
        return "".join(out)


class TTTNumpyCodec(Codec):
    """3x3 int8 boards indexed state[x][y] (reference test_games/tic_tac_toe_np.py)."""
    game_id = _lib.GAME_TTT
    name = "tic_tac_toe_np"

    def key(self, pos):
        if not isinstance(pos, np.ndarray) or pos.shape != (3, 3):
            raise ValueError("not a 3x3 board")
        v = pos.astype(np.int64)
        if ((v < 0) | (v > 2)).any():
            raise ValueError("cell out of range")
        return int(sum(int(v[x, y]) * 3 ** (x + 3 * y) for x in range(3) for y in range(3)))

    def pos(self, key):
        b = np.zeros((3, 3), dtype=np.int8)
        for i in range(9):
            b[i % 3, i // 3] = key % 3
            key //= 3
        return b


class TootCodec(Codec):
    """Latin-1 packed Toot-and-Otto positions (reference toot_and_otto_bitstring.py).

    key = the first 2A+16 bits (planes + hands).  The remaining bits must be the
    constant 1, zero padding, and a turn bit equal to the piece count mod 2.
    """
    game_id = _lib.GAME_TOOT
    name = "toot_and_otto"

    def __init__(self, length, height):
        self.L, self.H = int(length), int(height)
        self.A = self.L * self.H
        self.params = (self.L, self.H)
        self.nkey = 2 * self.A + 16
        self.nbits = -(-(self.nkey + 1) // 8) * 8

    def key(self, pos):
        if not isinstance(pos, str) or len(pos) != self.nbits // 8:
            raise ValueError("not a Toot position of this board")
        v = int.from_bytes(pos.encode("ISO-8859-1"), "big")
        key = v >> (self.nbits - self.nkey)
        tail = v & ((1 << (self.nbits - self.nkey)) - 1)
        pieces = bin((key >> 16) & ((1 << (2 * self.A)) - 1)).count("1")
        if tail != self._tail(pieces):
            raise ValueError("constant/padding/turn bits do not match")
        return key

    def _tail(self, pieces):
        width = self.nbits - self.nkey
        return (1 << (width - 1)) | (pieces & 1)

    def pos(self, key):
        pieces = bin((key >> 16) & ((1 << (2 * self.A)) - 1)).count("1")
        v = (key << (self.nbits - self.nkey)) | self._tail(pieces)
        return v.to_bytes(self.nbits // 8, "big").decode("ISO-8859-1")


class OthelloCodec(Codec):
    """Latin-1 packed Othello positions (reference othello_bit_new.py); key = all bits (8x8:
    144 bits, a Python int the context passes as 3 u64 words, include/gmsolve.h gm_key_words)."""
    game_id = _lib.GAME_OTHELLO
    name = "othello"

    def __init__(self, length, height):
        self.L, self.H = int(length), int(height)
        self.A = self.L * self.H
        self.params = (self.L, self.H)
        self.nbits = 2 * self.A + 16
        if self.nbits % 8:
            raise ValueError("board bits are not a whole number of bytes")

    def key(self, pos):
        if not isinstance(pos, str) or len(pos) != self.nbits // 8:
            raise ValueError("not an Othello position of this board")
        return int.from_bytes(pos.encode("ISO-8859-1"), "big")

    def pos(self, key):
        return key.to_bytes(self.nbits // 8, "big").decode("ISO-8859-1")


class SubtractCodec(Codec):
    """Nibble-packed heaps (test_games/subtraction.py, the synthetic config)."""
    game_id = _lib.GAME_SUBTRACT
    name = "subtraction"

    def __init__(self, heaps):
        self.heaps = int(heaps)
        self.params = (self.heaps,)

    def key(self, pos):
        if isinstance(pos, (bool, str, np.ndarray)) or not isinstance(pos, (int, np.integer)):
            raise ValueError("not a subtraction position")
        k = int(pos)
        if k < 0 or k >> (4 * self.heaps):
            raise ValueError("out of range")
        return k

    def pos(self, key):
        return int(key)


def _candidates(module):
    dims = (getattr(module, "length", None), getattr(module, "height", None))
    out = []
    if hasattr(module, "HEAPS"):
        out.append(SubtractCodec(module.HEAPS))
    out += [TTTStringCodec(), TTTNumpyCodec(), FourToOneCodec()]
    if dims[0] is not None and dims[1] is not None:
        for cls in (TootCodec, OthelloCodec):
            try:
                out.append(cls(*dims))
            except ValueError:
                pass
    return out


class HostDescriptor:
    """A context used only for gm_expand_host (no device work)."""

    def __init__(self, codec):
        self.codec = codec
        L = _lib.lib()
        params = (ctypes_i32 * max(1, len(codec.params)))(*codec.params)
        h = _lib.ctypes.c_void_p()
        _lib.check(L.gm_open(codec.game_id, params, len(codec.params), -1, _lib.ctypes.byref(h)))
        self.h = h
        self.words = L.gm_key_words(h)   # 3 for Othello 8x8 (keys past 64 bits)
        self._kids = (_lib.ctypes.c_uint64 * (64 * self.words))()
        self._key = (_lib.ctypes.c_uint64 * self.words)()

    def expand(self, key):
        L = _lib.lib()
        n, p, t = _lib.ctypes.c_int(), _lib.ctypes.c_int(), _lib.ctypes.c_int64()
        if self.words > 1:
            self._key[:] = _lib.int_to_words(key, self.words)
            _lib.check(L.gm_expand_host_key(self.h, self._key, self._kids, 64, _lib.ctypes.byref(n),
                                            _lib.ctypes.byref(p), _lib.ctypes.byref(t)))
            w = self.words
            return p.value, [_lib.words_to_int(self._kids[w * i:w * i + w]) for i in range(n.value)], t.value
        _lib.check(L.gm_expand_host(self.h, key, self._kids, 64, _lib.ctypes.byref(n),
                                    _lib.ctypes.byref(p), _lib.ctypes.byref(t)))
        return p.value, list(self._kids[:n.value]), t.value

    def initial(self):
        if self.words > 1:
            _lib.check(_lib.lib().gm_pack_initial_key(self.h, self._key))
            return _lib.words_to_int(self._key)
        k = _lib.ctypes.c_uint64()
        _lib.check(_lib.lib().gm_pack_initial(self.h, _lib.ctypes.byref(k)))
        return k.value

    def close(self):
        if self.h:
            _lib.lib().gm_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


ctypes_i32 = _lib.ctypes.c_int32


def verify(module, codec, root, samples=48, max_positions=600, seed=0):
    """Replay ``module`` against the descriptor from ``root``; True iff they agree.

    Checks, on a breadth-first prefix of the game graph and on random playouts:
    the primitive value, and the SET of child keys (gen_moves + do_move).
    """
    try:
        hd = HostDescriptor(codec)
    except _lib.GMError:
        return False
    try:
        rng = random.Random(seed)
        seen = set()

        def check(pos):
            k = codec.key(pos)
            prim, kids, _ = hd.expand(k)
            if module.primitive(pos) != prim:
                return None
            if prim != 4:
                return []
            children = [module.do_move(pos, m) for m in module.gen_moves(pos)]
            if sorted(codec.key(c) for c in children) != sorted(kids):
                return None
            return children

        frontier = [root]
        while frontier and len(seen) < max_positions:
            nxt = []
            for pos in frontier:
                k = codec.key(pos)
                if k in seen:
                    continue
                seen.add(k)
                kids = check(pos)
                if kids is None:
                    return False
                nxt.extend(kids)
                if len(seen) >= max_positions:
                    break
            frontier = nxt
        for _ in range(samples):
            pos = root
            for _depth in range(10000):
                kids = check(pos)
                if kids is None:
                    return False
                if not kids:
                    break
                pos = kids[rng.randrange(len(kids))]
        return True
    except (ValueError, TypeError, KeyError, IndexError, AttributeError, _lib.GMError):
        return False
    finally:
        hd.close()


EXHAUSTIVE_MAX = int(os.environ.get("GM_BIND_EXHAUSTIVE_MAX", 1_000_000))


def verify_exhaustive(module, codec, root, max_positions=None):
    """Every position reachable from ``root`` checked against the descriptor: the
    primitive value and the set of child keys.  True iff they all agree; False at
    the first difference or once more than ``max_positions`` positions are reached
    (then the match is not certain)."""
    max_positions = EXHAUSTIVE_MAX if max_positions is None else max_positions
    try:
        hd = HostDescriptor(codec)
    except _lib.GMError:
        return False
    try:
        k0 = codec.key(root)
        seen = {k0}
        frontier = [root]
        while frontier:
            nxt = []
            for pos in frontier:
                prim, kids, _ = hd.expand(codec.key(pos))
                if module.primitive(pos) != prim:
                    return False
                if prim != 4:
                    continue
                children = [module.do_move(pos, m) for m in module.gen_moves(pos)]
                ck = [codec.key(c) for c in children]
                if sorted(ck) != sorted(kids):
                    return False
                for c, k in zip(children, ck):
                    if k not in seen:
                        seen.add(k)
                        nxt.append(c)
                if len(seen) > max_positions:
                    return False
            frontier = nxt
        return True
    except (ValueError, TypeError, KeyError, IndexError, AttributeError, _lib.GMError):
        return False
    finally:
        hd.close()


def identify(module, root=None, exhaustive_max=None):
    """Return the codec whose device descriptor reproduces ``module`` (or None).

    Binding must be certain (a plugin that differs from a descriptor only in deep
    or rare positions would otherwise be solved with the descriptor's rules, a
    wrong answer with no error), so a codec is returned only when
      * the plugin's code fingerprint (gamesmanmpi_amd/fingerprint.py) is one of the
        plugin files that descriptor was written from -- the reference's own
        test_games files or this repo's rewrites -- and a sample of positions
        agrees (the board dimensions and heap count are module parameters); or
      * every position reachable from ``root``, at most ``exhaustive_max``
        (GM_BIND_EXHAUSTIVE_MAX, default 10^6), agrees with the descriptor.
    Otherwise the plugin goes to the explicit-graph engine (gamesmanmpi_amd/graph.py).
    Reference: the launcher's plugin check, solver_launcher.py:70-81."""
    from . import fingerprint as fp
    if root is None:
        root = module.initial_position()
    cands = []
    for codec in _candidates(module):
        try:
            codec.key(root)
        except (ValueError, TypeError, OverflowError):
            continue
        cands.append(codec)
    mine = fp.known().get(fp.fingerprint(module))
    for codec in cands:
        if mine and mine["codec"] == codec.name and verify(module, codec, root):
            return codec
    for codec in cands:
        if verify(module, codec, root) and verify_exhaustive(module, codec, root, exhaustive_max):
            return codec
    return None
