"""LDS bank model of the box engine's image (csrc/dense_box.hip), development aid.

    python tools/lds_bank_model.py [PITCH[/ASTRIDE[/ZSLOT]][x] ...]

(e.g. 68/16 = round 3, 76/20/19 = round 4's layout, 68/16x = pitch 68 with the 16-B chunk
index XOR-swizzled by the p-row, the verdict r03 suggestion)

Counts LDS-array cycles per group for every LDS access of the kernel, by the CDNA4 rules
of MI355X_MICROARCH.md section LDS: ds_read_b32 / ds_write_b32 in two 32-lane groups
(bank = dword mod 32, a write costs at least 4), ds_read_b128 in four 16-lane groups
(bank = dword mod 64), ds_write_b128 in eight 8-lane groups (bank = dword mod 32, at
least 13); each extra distinct dword on a bank within a group adds a cycle.

Image: position (A = a0 + 4 p, B) at dword PITCH p + ASTRIDE a0 + B; the walk's lane
(a0 = lane & 3, b = lane >> 2) starts at d = b0 + b1 + 2 (b2 + b3) + a0 and per step
writes its code and reads its fold value and its b2 / b3 neighbours' codes (4 / 8
dwords lower, or a zero slot: PITCH p + 64 + a0 of the row padding, or with ZSLOT the
one slot PITCH p + ZSLOT of the p-row).  With the swizzle, B's 16-B chunk B >> 2 is
stored at chunk (B >> 2) ^ (p & 3).
"""
import collections
import sys

# ds_read_b128 lane groups (MI355X_MICROARCH.md)
RG128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
         list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
RG128 += [[x + 32 for x in g] for g in RG128]


def b32(addrs, write=False):
    c = 0
    for g in (range(0, 32), range(32, 64)):
        banks = collections.defaultdict(set)
        for lane in g:
            if addrs[lane] is not None:
                banks[addrs[lane] % 32].add(addrs[lane])
        c += max((len(v) for v in banks.values()), default=1)
    return max(4, c) if write else c


def b128_read(addrs):
    c = 0
    for g in RG128:
        banks = collections.defaultdict(set)
        for lane in g:
            for e in range(4):
                banks[(addrs[lane] + e) % 64].add(addrs[lane] + e)
        c += max(len(v) for v in banks.values())
    return c


def b128_write(addrs):
    c = 0
    for g0 in range(0, 64, 8):
        banks = collections.defaultdict(set)
        for lane in range(g0, g0 + 8):
            for e in range(4):
                banks[(addrs[lane] + e) % 32].add(addrs[lane] + e)
        c += max(len(v) for v in banks.values())
    return max(13, c)


def model(pitch, astride=16, zslot=None, swz=False):
    def addr(A, B):
        p = A >> 2
        c = (B >> 2) ^ (p & 3) if swz else B >> 2
        return pitch * p + astride * (A & 3) + 4 * c + (B & 3)

    def zero(p, a0):
        return pitch * p + (zslot if zslot is not None else 64 + a0)

    dmax = 2 + 4 + 3
    walk = 0
    for T in range(64 + dmax):
        F, C2, C3 = [], [], []
        for lane in range(64):
            a0, b = lane & 3, (lane >> 2) & 15
            d = bin(b & 3).count("1") + 2 * bin(b & 12).count("1") + a0
            p = T - d
            if 0 <= p < 64:
                F.append(addr(a0 + 4 * p, b))
                C2.append(addr(a0 + 4 * p, b - 4) if b & 4 else zero(p, a0))
                C3.append(addr(a0 + 4 * p, b - 8) if b & 8 else zero(p, a0))
            else:   # idle step: the lane's dummy slot
                F.append(100000 + lane)
                C2.append(100000 + lane)
                C3.append(100000 + lane)
        walk += b32(F, True) + b32(F) + b32(C2) + b32(C3)
    fold = 0
    for i in range(4):   # phase-1 writes and the store's reads: rows m = lane + 64 i
        for q in range(4):
            rows = [addr(lane + 64 * i, 4 * q) for lane in range(64)]
            fold += b128_write(rows) + b128_read(rows)
    for i in range(3):   # phase 2: rows a_i = 0, 1 of heaps 0-2, read and written
        for r in (0, 1):
            rows = []
            for lane in range(64):
                lo, hi = lane & ((1 << (2 * i)) - 1), (lane >> (2 * i)) << (2 * i + 2)
                rows.append(lo | (r << (2 * i)) | hi)
            for q in range(4):
                a = [addr(A, 4 * q) for A in rows]
                fold += b128_read(a) + b128_write(a)
    return walk, fold


def main():
    specs = sys.argv[1:] or [str(p) for p in range(68, 79)]
    ideal_walk = (64 + 9) * (4 + 2 + 2 + 2)
    print("layout        walk  fold+store  total   (conflict-free walk: %d)" % ideal_walk)
    for spec in specs:
        swz = spec.endswith("x")
        parts = [int(x) for x in spec.rstrip("x").split("/")]
        w, f = model(parts[0], parts[1] if len(parts) > 1 else 16, parts[2] if len(parts) > 2 else None, swz)
        print("%-12s %5d %11d %6d" % (spec, w, f, w + f))


if __name__ == "__main__":
    main()
