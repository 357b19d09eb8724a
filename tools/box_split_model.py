#!/usr/bin/env python3
"""Model of two multi-GPU designs for the 8-heap subtraction game (config 5, 2^32 positions)
on the box engine (csrc/dense_box.hip), VERDICT r04 item 1.  CPU only, numpy.

    python tools/box_split_model.py [--batch 4] [--lat-us 15] [--link-gbs 64]

(a) DISJOINT BOX SPLIT, no symmetry in the computation: rank bit a = [c_d >= thr] for the
    split heap d of axis a (box coordinates c_0..c_3 in 0..3, c_4..c_7 in 0..7; thr = 2 / 4),
    every box computed by exactly one rank.  A child box lies one box step below its parent
    along one heap, so a child crosses at most one axis, always downwards: the upper rank of
    axis a needs the boundary layer c_d = thr - 1 of its lower neighbour (A heap: the child
    box's top two A layers, 2 KiB; B heap: the whole 4 KiB box).  Optional symmetric fill:
    the boundary box C is the transposition (d p) of a box the upper rank computes itself in
    the same box-tier when some unsplit heap p of the same kind has c_p >= thr; then nothing
    crosses the link for C (the kernel reads the child through the transposition).  The
    exchange is batched: batch j = box-tiers [jB, jB+B), its message carries the lower
    rank's boundary boxes of box-tiers [jB-1, jB+B-2], packed after that rank's tier jB+B-2.
(b) H-QUOTIENT AT N = 1 AND N > 1: compute only F, one box per orbit of H = <rotate heaps
    0-3> x <swap 4<->5, 6<->7> (|H| = 8; 145,600 boxes incl. ties), then write the other
    members of every orbit as images; at N > 1 the ranks split F by box coordinates and
    exchange F's cross-rank children per batch as in (a), and each writes its part's images.

Time model, per rank on one MI355X: a box-tier launch of n groups (box pairs) costs
max(7.0 us, n / 172 per us) + 5.5 us -- fitted to the round-4 measurements of the orbit
plan's tier launches (3.31 / 1.88 / 1.16 / 0.77 ms at G = 1 / 2 / 4 / 8 for its exact
per-tier counts, profiles/r04n_box_shard_time.txt), within 1.4 % at every G.  A message
costs lat + bytes / link (one xGMI link per rank pair, one direction used), its pack and
unpack 3 us + bytes / 3 TB/s each, on the axis's exchange stream.  The schedule is the op
list's: a rank's compute stream runs its batches in order; batch j first waits for the
unpack of every message X_j it receives.
"""
import argparse
import json
import math

import numpy as np

NB = 1 << 20
C = np.arange(NB, dtype=np.int64)
COORD = [(C >> (2 * i)) & 3 for i in range(4)] + [(C >> (8 + 3 * j)) & 7 for j in range(4)]
TIER = sum(COORD)
THR = [2] * 4 + [4] * 4
LIM = [3] * 4 + [7] * 4
UNIT = [1 << (2 * i) for i in range(4)] + [1 << (8 + 3 * j) for j in range(4)]

AXES = {2: [3], 4: [3, 7], 8: [2, 3, 7]}     # split heaps per world size (A heaps 0-3, B heaps 4-7)


def launch_us(groups):
    g = np.asarray(groups, dtype=np.float64)
    return np.where(g > 0, np.maximum(7.0, g / 172.0) + 5.5, 0.0)


def owner(axes):
    r = np.zeros(NB, dtype=np.int64)
    for a, d in enumerate(axes):
        r |= (COORD[d] >= THR[d]).astype(np.int64) << a
    return r


def halo(axes, fill):
    """Per axis: the boundary boxes that cross the link (bool mask over box ids) and bytes/box."""
    out = []
    split = set(axes)
    for a, d in enumerate(axes):
        bnd = COORD[d] == THR[d] - 1
        send = bnd.copy()
        if fill:
            same = range(4) if d < 4 else range(4, 8)
            for p in same:
                if p == d or p in split:
                    continue
                send &= ~(COORD[p] >= THR[d])
        out.append((send, 2048 if d < 4 else 4096, bnd))
    return out


def batches(ntiers, B):
    nb = (ntiers + B - 1) // B
    return [(max(0, j * B - 1), min(ntiers - 2, j * B + B - 2)) for j in range(nb)]


def simulate(per_rank_tier_groups, msgs, G, B, lat_us, link_gbs, ntiers=41):
    """per_rank_tier_groups[r][t]; msgs[(a, j)] -> bytes from each lower rank to its upper
    neighbour (per rank pair: dict lower_rank -> bytes).  Returns per-rank end times (us)."""
    g = G.bit_length() - 1
    bl = batches(ntiers, B)
    nbat = len(bl)
    tier_end = np.zeros((G, ntiers))
    end = np.zeros(G)
    x_free = np.zeros((G, max(1, g)))      # exchange stream availability, per rank and axis
    arrive = {}
    # ranks in an order where every lower neighbour precedes: by popcount then value
    order = sorted(range(G), key=lambda r: (bin(r).count("1"), r))
    for r in order:
        t_s = 0.0
        for j in range(nbat):
            start = t_s
            for a in range(g):
                if (r >> a) & 1:
                    k = (a, j, r ^ (1 << a))
                    if k in arrive:
                        start = max(start, arrive[k])
            t = start
            for tt in range(j * B, min(ntiers, j * B + B)):
                t += float(launch_us(per_rank_tier_groups[r][tt]))
                tier_end[r, tt] = t
                # lower side: message X_j' packed after tier hi_j'
                for jj, (lo, hi) in enumerate(bl):
                    if hi != tt:
                        continue
                    for a in range(g):
                        if (r >> a) & 1:
                            continue
                        nbytes = msgs.get((a, jj), {}).get(r, 0)
                        if not nbytes:
                            continue
                        p0 = max(tier_end[r, tt], x_free[r, a])
                        pack = 3.0 + nbytes / 3e6
                        xfer = lat_us + nbytes / (link_gbs * 1e3)
                        unpack = 3.0 + nbytes / 3e6
                        x_free[r, a] = p0 + pack + xfer
                        arrive[(a, jj, r)] = p0 + pack + xfer + unpack
            t_s = t
        end[r] = t_s
    return end


def design_a(G, B, lat_us, link_gbs, fill, axes=None):
    if G == 1:
        groups = [(np.bincount(TIER, minlength=41) + 1) // 2]
        return {"G": 1, "ms": round(float(launch_us(groups[0]).sum()) / 1000, 3), "boxes_per_rank": [NB]}
    axes = axes or AXES[G]
    own = owner(axes)
    per = []
    for r in range(G):
        cnt = np.bincount(TIER[own == r], minlength=41)
        per.append((cnt + 1) // 2)
    H = halo(axes, fill)
    bl = batches(41, B)
    msgs = {}
    sent_total = 0
    nmsg = 0
    for a, (send, bpb, bnd) in enumerate(H):
        for j, (lo, hi) in enumerate(bl):
            m = send & (TIER >= lo) & (TIER <= hi)
            if not m.any():
                continue
            by = np.bincount(own[m], minlength=G) * bpb
            msgs[(a, j)] = {r: int(by[r]) for r in range(G) if by[r]}
            nmsg += sum(1 for r in range(G) if by[r])
            sent_total += int(by.sum())
    end = simulate(per, msgs, G, B, lat_us, link_gbs)
    per_link = {}
    for (a, j), d in msgs.items():
        for r, b in d.items():
            per_link[(a, r)] = per_link.get((a, r), 0) + b
    compute = [float(launch_us(p).sum()) / 1000 for p in per]
    return {"G": G, "axes": axes, "fill": fill, "ms": round(float(end.max()) / 1000, 3),
            "per_rank_ms": [round(float(e) / 1000, 3) for e in end],
            "compute_only_ms": [round(c, 3) for c in compute],
            "boxes_per_rank": [int((own == r).sum()) for r in range(G)],
            "tiers_per_rank": [int((np.bincount(TIER[own == r], minlength=41) > 0).sum()) for r in range(G)],
            "halo_boxes_per_axis": [int(h[2].sum()) for h in H],
            "sent_boxes_per_axis": [int(h[0].sum()) for h in H],
            "max_link_mib": round(max(per_link.values()) / 2**20, 1) if per_link else 0.0,
            "sent_mib_total": round(sent_total / 2**20, 1), "messages": nmsg,
            "work_vs_one_gpu": 1.0}


def orbit_F():
    """F: the least member of every H-orbit in the B-first order (csrc/dense_box.hip round 4)."""
    def rot(b, k):
        f = b & 0xFF
        f = ((f | (f << 8)) >> (8 - 2 * k)) & 0xFF
        return (b & ~0xFF) | f

    def tau(b):
        x = ((b >> 3) ^ b) & 0x1C700
        return b ^ x ^ (x << 3)

    def ordk(b):
        o = np.zeros_like(b)
        for n in range(8):
            d = 4 + n if n < 4 else n - 4
            o = (o << 3) | ((b >> (2 * d)) & 3 if d < 4 else (b >> (8 + 3 * (d - 4))) & 7)
        return o
    imgs = [rot(C, k) if e == 0 else tau(rot(C, k)) for k in range(4) for e in range(2)]
    ords = np.stack([ordk(x) for x in imgs])
    return ords[0] == ords.min(0)


def design_b(G, B, lat_us, link_gbs, write_tbs=5.0, overlap=0.5):
    """(b): F computed (split by coordinates at N > 1, exchange as in (a) without fill: F is
    not closed under the transpositions), images written (4 GiB minus F), overlap = the share
    of the image writes hidden under the latency-bound chain."""
    F = orbit_F()
    nF = int(F.sum())
    img_bytes = (NB - nF) * 4096
    if G == 1:
        cnt = (np.bincount(TIER[F], minlength=41) + 1) // 2
        comp = float(launch_us(cnt).sum())
        w = img_bytes / (write_tbs * 1e6)
        return {"G": 1, "F_boxes": nF, "ms": round((comp + (1 - overlap) * w) / 1000, 3),
                "compute_ms": round(comp / 1000, 3), "image_write_ms": round(w / 1000, 3),
                "work_vs_one_gpu_a": round(nF / NB, 3)}
    axes = AXES[G]
    own = owner(axes)
    per = [(np.bincount(TIER[F & (own == r)], minlength=41) + 1) // 2 for r in range(G)]
    H = halo(axes, False)
    msgs = {}
    for a, (send, bpb, bnd) in enumerate(H):
        # a boundary box is sent if it is in F or read through an image of F -- bound by (a)'s halo
        for j, (lo, hi) in enumerate(batches(41, B)):
            m = bnd & F & (TIER >= lo) & (TIER <= hi)
            if m.any():
                by = np.bincount(own[m], minlength=G) * bpb
                msgs[(a, j)] = {r: int(by[r]) for r in range(G) if by[r]}
    end = simulate(per, msgs, G, B, lat_us, link_gbs)
    w = img_bytes / G / (write_tbs * 1e6)
    t = float(end.max()) + (1 - overlap) * w
    return {"G": G, "F_boxes_per_rank": [int((F & (own == r)).sum()) for r in range(G)],
            "ms": round(t / 1000, 3), "chain_ms": round(float(end.max()) / 1000, 3),
            "image_write_ms_per_rank": round(w / 1000, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--lat-us", type=float, default=15.0)
    ap.add_argument("--link-gbs", type=float, default=64.0)
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    print("# (a) disjoint box split, batch %d, message latency %.0f us, link %.0f GB/s one way"
          % (a.batch, a.lat_us, a.link_gbs))
    base = None
    for fill in (True, False):
        for G in (1, 2, 4, 8):
            r = design_a(G, a.batch, a.lat_us, a.link_gbs, fill)
            base = base or r["ms"]
            r["speedup"] = round(base / r["ms"], 2)
            print(json.dumps(r))
    print("# (a) axis choices at G = 4, 8 (fill on)")
    for G, axes in ((2, [7]), (4, [6, 7]), (4, [2, 3]), (8, [3, 6, 7]), (8, [1, 2, 3]), (8, [5, 6, 7])):
        r = design_a(G, a.batch, a.lat_us, a.link_gbs, True, axes)
        print(json.dumps({k: r[k] for k in ("G", "axes", "ms", "max_link_mib", "tiers_per_rank")}))
    print("# (a) sensitivity at G = 8 (fill on): latency x link bandwidth")
    for lat in (5.0, 15.0, 30.0):
        for bw in (40.0, 64.0, 100.0):
            r = design_a(8, a.batch, lat, bw, True)
            print(json.dumps({"lat_us": lat, "link_gbs": bw, "ms": r["ms"], "speedup": round(base / r["ms"], 2)}))
    print("# (a) batch size at G = 8 (fill on)")
    for B in (1, 2, 4, 8):
        r = design_a(8, B, a.lat_us, a.link_gbs, True)
        print(json.dumps({"batch": B, "ms": r["ms"], "messages": r["messages"]}))
    print("# (b) H-quotient at N = 1 and N > 1 (image writes at 5 TB/s, half hidden under the chain)")
    for G in (1, 2, 4, 8):
        print(json.dumps(design_b(G, a.batch, a.lat_us, a.link_gbs)))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
