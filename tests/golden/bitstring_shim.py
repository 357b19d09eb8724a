"""Minimal stand-in for the third-party ``bitstring.BitArray`` (golden generation only).

The reference's Toot-and-Otto and Othello plugins build positions with
``bitstring.BitArray`` (unpinned version: not in ``requirements.txt``;
``run_savio.sh:38`` installs it unversioned).  The package is absent here, so this
shim restates the documented semantics of the subset those two plugins use:

* bits are MSB-first; ``BitArray('0b0110')``, ``BitArray()``;
* ``a * n`` repeats; ``append`` concatenates;
* ``a[i]`` (negative allowed) -> bool; ``a[i:j]`` -> BitArray copy;
* ``a[i] = bool``; ``a[i:j] = BitArray`` (same length) or ``= int`` (encoded in
  the slice length, unsigned when >= 0, two's complement when < 0);
* ``.int`` two's-complement value of the whole array (getter and setter);
* ``.bytes`` MSB-first (length must be a whole number of bytes; getter and setter);
* ``|`` and ``==``.

It is used only by ``tests/golden/make_golden.py`` in the survey/build container
and never ships with the solver.
"""


class BitArray:
    __slots__ = ("_v", "_n")

    def __init__(self, auto=None, *, _v=0, _n=0):
        if auto is None:
            self._v, self._n = _v, _n
        elif isinstance(auto, str):
            if not auto.startswith("0b"):
                raise ValueError("only '0b...' literals are supported")
            digits = auto[2:]
            self._v = int(digits, 2) if digits else 0
            self._n = len(digits)
        elif isinstance(auto, BitArray):
            self._v, self._n = auto._v, auto._n
        else:
            raise TypeError("unsupported initialiser %r" % (auto,))

    @classmethod
    def _make(cls, v, n):
        return cls(_v=v & ((1 << n) - 1) if n else 0, _n=n)

    def __len__(self):
        return self._n

    @property
    def len(self):
        return self._n

    def _bit(self, i):
        return (self._v >> (self._n - 1 - i)) & 1

    def __mul__(self, times):
        v, n = 0, 0
        for _ in range(times):
            v = (v << self._n) | self._v
            n += self._n
        return BitArray._make(v, n)

    def append(self, other):
        other = other if isinstance(other, BitArray) else BitArray(other)
        self._v = (self._v << other._n) | other._v
        self._n += other._n

    def _norm(self, key):
        start, stop, step = key.indices(self._n)
        if step != 1:
            raise ValueError("stepped slices are not supported")
        return start, max(start, stop)

    def __getitem__(self, key):
        if isinstance(key, slice):
            a, b = self._norm(key)
            width = b - a
            return BitArray._make(self._v >> (self._n - b), width)
        if key < 0:
            key += self._n
        if not 0 <= key < self._n:
            raise IndexError(key)
        return bool(self._bit(key))

    def __setitem__(self, key, value):
        if isinstance(key, slice):
            a, b = self._norm(key)
            width = b - a
            if isinstance(value, int) and not isinstance(value, bool):
                if value >= 0:
                    if value >> width:
                        raise ValueError("value does not fit the slice")
                    bits = value
                else:
                    if value < -(1 << (width - 1)):
                        raise ValueError("value does not fit the slice")
                    bits = value & ((1 << width) - 1)
            else:
                value = value if isinstance(value, BitArray) else BitArray(value)
                if value._n != width:
                    raise ValueError("slice replacement of a different length")
                bits = value._v
            shift = self._n - b
            mask = ((1 << width) - 1) << shift
            self._v = (self._v & ~mask) | (bits << shift)
            return
        if key < 0:
            key += self._n
        if not 0 <= key < self._n:
            raise IndexError(key)
        mask = 1 << (self._n - 1 - key)
        if value:
            self._v |= mask
        else:
            self._v &= ~mask

    @property
    def int(self):
        if self._n == 0:
            raise ValueError("empty bitstring has no int value")
        if self._v >> (self._n - 1):
            return self._v - (1 << self._n)
        return self._v

    @int.setter
    def int(self, value):
        lo, hi = -(1 << (self._n - 1)), (1 << (self._n - 1)) - 1
        if not lo <= value <= hi:
            raise ValueError("int %d does not fit %d bits" % (value, self._n))
        self._v = value & ((1 << self._n) - 1)

    @property
    def bytes(self):
        if self._n % 8:
            raise ValueError("not a whole number of bytes")
        return self._v.to_bytes(self._n // 8, "big")

    @bytes.setter
    def bytes(self, data):
        self._v = int.from_bytes(data, "big")
        self._n = 8 * len(data)

    def __or__(self, other):
        if self._n != other._n:
            raise ValueError("length mismatch")
        return BitArray._make(self._v | other._v, self._n)

    def __eq__(self, other):
        other = other if isinstance(other, BitArray) else BitArray(other)
        return self._n == other._n and self._v == other._v

    def __hash__(self):
        return hash((self._v, self._n))
