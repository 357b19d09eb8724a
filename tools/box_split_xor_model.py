#!/usr/bin/env python3
"""Tier-ordered model of two box partitions over G ranks (development aid).

    python tools/box_split_xor_model.py

'halves' is the split dist_box.hip builds (rank bit a = [c_h >= threshold] for one heap per
axis: crossings one way, lower -> upper); 'xor' gives every rank work at every tier (rank bit
a = [c_A >= 2] XOR [c_B >= 4] for one A and one B heap per axis) at the price of crossings both
ways, so each rank's tier t waits for its axis peers' tier t - 1 every tier.  A rank's tier
lasts max(groups / rate, floor) us (rate = the one-GPU thick-tier throughput, 169 groups/us;
floor = the lone-group latency) and starts `lat` us after the tiers it reads.  Pure numpy over
the 2^20 boxes; no GPU, no library."""
import numpy as np

A, B = np.arange(4), np.arange(8)
C = np.stack([g.ravel() for g in np.meshgrid(A, A, A, A, B, B, B, B, indexing="ij")], 1)
TIER = C.sum(1)
T = 41


def halves(G):
    r = np.zeros(len(C), int)
    for a, (h, t) in enumerate({2: [(3, 2)], 4: [(3, 2), (7, 4)], 8: [(2, 2), (3, 2), (7, 4)]}[G]):
        r |= (C[:, h] >= t).astype(int) << a
    return r


def xor(G):
    r = np.zeros(len(C), int)
    for a, (h1, h2) in enumerate({2: [(3, 7)], 4: [(3, 7), (2, 6)], 8: [(3, 7), (2, 6), (1, 5)]}[G]):
        r |= ((C[:, h1] >= 2) ^ (C[:, h2] >= 4)).astype(int) << a
    return r


def makespan_ms(r, G, twoway, rate=169.0, lat=0.0, floor=0.0):
    groups = np.array([(np.bincount(TIER[r == k], minlength=T) + 1) // 2 for k in range(G)])
    end = np.zeros((G, T))
    for t in range(T):
        for k in range(G):
            st = end[k, t - 1] if t else 0.0
            for ax in range(G.bit_length() - 1):
                if t and (twoway or (k >> ax) & 1):
                    st = max(st, end[k ^ (1 << ax), t - 1] + lat)
            n = groups[k, t]
            end[k, t] = st + (max(n / rate, floor) if n else 0.0)
    return end[:, -1].max() / 1000


def main():
    one = ((np.bincount(TIER, minlength=T) + 1) // 2).sum() / 169.0 / 1000
    print("one GPU at the thick-tier rate: %.3f ms" % one)
    for G in (2, 4, 8):
        for lat, floor in ((0, 0), (3, 8), (5, 8), (5, 12), (10, 12), (20, 8)):
            mh, mx = makespan_ms(halves(G), G, False, lat=lat, floor=floor), makespan_ms(xor(G), G, True, lat=lat, floor=floor)
            print("G=%d hop %4.1f us floor %4.1f us: halves %.3f ms (%.2fx)  xor %.3f ms (%.2fx)"
                  % (G, lat, floor, mh, one / mh, mx, one / mx))


if __name__ == "__main__":
    main()
