"""CPU checks of the split box solve (csrc/dist_box.hip): plans, schedule, gloo ranks.
Test infrastructure.

The plans come from the product: ``gm_box_plan`` runs the host code gm_solve uses
(bx_shape / bx_plan / bx_build_ops) without touching a GPU.

``simulate`` executes every rank's RCCL-mode op list under the semantics that path relies on
-- one FIFO per HIP stream (S, X[axis]), a hipStreamWaitEvent bound to the record of that
event enqueued before it, the k-th ncclSend from rank s to rank d on an axis matching the
k-th ncclRecv at d from s -- in a random interleaving of whatever is ready, and tracks which
boxes each rank holds: it fails on a deadlock, on a tier launch that reads a child box the
rank neither computed nor unpacked (or reads a fill source it did not compute), on a send of
a message whose boxes are not all computed yet (the tier kernel writes a box's message slots
as it computes it), and on sender / receiver lists that disagree.

``gloo_rank`` runs one rank's op list as a host program over torch.distributed (gloo): the
same messages, peers and order as RCCL mode, the oracle's codes as the payload, the rows a
message entry carries chosen as the tier kernel's halo store (bx_store) does.
"""
import random
from collections import defaultdict, deque

import numpy as np

from gamesmanmpi_amd import _lib

BOP_TIER, BOP_PACK, BOP_UNPACK, BOP_SEND, BOP_RECV, BOP_RECORD, BOP_WAIT = range(7)
BEV_DONE, BEV_PACKED = range(2)
FULL = 0xFFFFFFFF


def coords(b):
    b = np.asarray(b, dtype=np.int64)
    return [(b >> (2 * i)) & 3 for i in range(4)] + [(b >> (8 + 3 * j)) & 7 for j in range(4)]


def unit(d):
    return 1 << (2 * d) if d < 4 else 1 << (8 + 3 * (d - 4))


def box_of_key(key):
    key = np.asarray(key, dtype=np.int64)
    b = np.zeros_like(key)
    for i in range(4):
        b |= ((key >> (4 * i + 2)) & 3) << (2 * i)
    for j in range(4):
        b |= ((key >> (16 + 4 * j + 1)) & 7) << (8 + 3 * j)
    return b


def region(root):
    lim = coords(box_of_key(root))
    b = np.arange(1 << 20, dtype=np.int64)
    c = coords(b)
    ok = np.ones(len(b), bool)
    for i in range(8):
        ok &= c[i] <= lim[i]
    return b[ok]


def tier(b):
    return sum(coords(b))


def load_plan(world, rank, root=FULL, batch=4, symmetry=1, split=0, transport=0):
    kw = dict(root=root, batch=batch, symmetry=symmetry, split=split)
    P = {"rank": rank}
    sh = _lib.box_plan(world, rank, _lib.BOXPLAN_SHAPE, **kw).astype(np.int64)
    P["G"], P["g"], P["ntiers"], P["batch"], P["nbatch"], P["split"], P["fill"] = sh[:7].tolist()
    P["axes"] = [tuple(sh[7 + 4 * a:11 + 4 * a].tolist()) for a in range(3)]
    P["halo"] = _lib.box_plan(world, rank, _lib.BOXPLAN_HALO, **kw).astype(np.int64).reshape(-1, 2)
    for name, what in (("boxes", _lib.BOXPLAN_BOXES), ("fills", _lib.BOXPLAN_FILLS), ("off", _lib.BOXPLAN_TIER_OFF),
                       ("own", _lib.BOXPLAN_OWN), ("srcs", _lib.BOXPLAN_SRCS), ("counts", _lib.BOXPLAN_COUNTS)):
        P[name] = _lib.box_plan(world, rank, what, **kw).astype(np.int64)
    P["srcs"] = P["srcs"].reshape(-1, 8)
    P["send"], P["recv"] = [], []
    for a in range(3):
        P["send"].append((_lib.box_plan(world, rank, _lib.BOXPLAN_SEND_OFF, axis=a, **kw).astype(np.int64),
                          _lib.box_plan(world, rank, _lib.BOXPLAN_SEND, axis=a, **kw).astype(np.int64)))
        P["recv"].append((_lib.box_plan(world, rank, _lib.BOXPLAN_RECV_OFF, axis=a, **kw).astype(np.int64),
                          _lib.box_plan(world, rank, _lib.BOXPLAN_RECV, axis=a, **kw).astype(np.int64)))
    P["ops"] = _lib.box_plan(world, rank, _lib.BOXPLAN_OPS, transport=transport, **kw).astype(np.int64).reshape(-1, 6)
    P["direct"] = transport == 1   # the IPC transport: the sender's tier kernel writes the receiver's table
    return P


def plans(world, root=FULL, **kw):
    return [load_plan(world, r, root, **kw) for r in range(world)]


def seg(offdata, j):
    off, data = offdata
    if j < 0 or j + 1 >= len(off):
        return data[:0]
    return data[off[j]:off[j + 1]]


def entry_rows(e):
    """Rows (A indices) a message entry carries, in message order (bx_store / box_unpack_kernel)."""
    code = int(e) >> 20
    if code == 0:
        return np.arange(256)
    i2 = 2 * (code - 1)
    t = np.arange(128)
    return (t & ((1 << i2) - 1)) | ((2 | ((t >> i2) & 1)) << i2) | ((t >> (i2 + 1)) << (i2 + 2))


def fill_code(fill, d):
    return (int(fill) >> (4 * d)) & 15


def transposed_heaps(fill, d):
    """Heaps (q, p) of the transposition the child along heap d is read through, or None."""
    c = fill_code(fill, d)
    if d < 4:
        q, p = c >> 2, c & 3
        return None if q == p else (q, p)
    if c == 0:
        return None
    pairs = [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]
    q, p = pairs[c - 1]
    return 4 + q, 4 + p


def swap_box(b, q, p):
    c = coords(b)
    c[q], c[p] = c[p], c[q]
    out = 0
    for i in range(4):
        out |= int(c[i]) << (2 * i)
    for j in range(4):
        out |= int(c[4 + j]) << (8 + 3 * j)
    return out


class SimError(AssertionError):
    pass


PAIRS = np.array([(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)], np.int64)


def swap_boxes(b, q, p):
    """Boxes b with the coordinates of heaps q and p exchanged (elementwise; q, p of one kind)."""
    b, q, p = (np.asarray(x, np.int64) for x in (b, q, p))
    sq = np.where(q < 4, 2 * q, 8 + 3 * (q - 4))
    sp = np.where(p < 4, 2 * p, 8 + 3 * (p - 4))
    m = np.where(q < 4, 3, 7)
    fq, fp = (b >> sq) & m, (b >> sp) & m
    return (b & ~(m << sq) & ~(m << sp)) | (fq << sp) | (fp << sq)


def direction_reads(P, d):
    """For every computed box with a child along heap d: (box index, child C, source read,
    swapped?) -- the kernel's read of that child (dense_box.hip bx_issue), vectorised."""
    boxes = P["boxes"]
    c = coords(boxes)
    idx = np.nonzero(c[d] >= 1)[0]
    C = boxes[idx] - unit(d)
    src = P["srcs"][idx, d]
    code = (P["fills"][idx] >> (4 * d)) & 15
    if d < 4:
        q, p = code >> 2, code & 3
        sw = q != p
    else:
        sw = code != 0
        pr = PAIRS[np.maximum(code - 1, 0)]
        q, p = 4 + pr[:, 0], 4 + pr[:, 1]
    return idx, C, src, sw, q, p


def received_keys(P):
    """batch << 28 | code << 20 | box of every entry the rank receives."""
    ks = []
    for a in range(3):
        offs, ent = P["recv"][a]
        for j in range(len(offs) - 1):
            ks.append((np.int64(j) << 28) | ent[offs[j]:offs[j + 1]].astype(np.int64))
    return np.unique(np.concatenate(ks)) if ks else np.zeros(0, np.int64)


def check_reads(P, received=None):
    """Every child read of every computed box resolves (the kernel's contract): an own box of
    the tier below, a same-kind heap transposition of one (the fill), or an entry of the
    parent's batch's halo message (a whole box, or for an A-heap child its two top layers)."""
    boxes, off = P["boxes"], P["off"]
    tier_of = np.full(1 << 20, -1, np.int64)
    tier_of[boxes] = np.repeat(np.arange(len(off) - 1), np.diff(off))
    T = tier_of[boxes]
    rk = received_keys(P)
    for d in range(8):
        idx, C, src, sw, q, p = direction_reads(P, d)
        t = T[idx]
        if sw.any():
            exp = swap_boxes(C[sw], q[sw], p[sw])
            bad = (src[sw] != exp) | (exp == C[sw]) | (tier_of[exp] != t[sw] - 1)
            if bad.any():
                i = np.nonzero(bad)[0][0]
                raise SimError("rank %d box %#x dir %d: fill source %#x is not an own box of the tier below, "
                               "or not the transposition (%d %d) of %#x" % (P["rank"], boxes[idx[sw][i]], d,
                                                                          src[sw][i], q[sw][i], p[sw][i], C[sw][i]))
            if ((q[sw] < 4) != (d < 4)).any():
                raise SimError("rank %d: a child along heap %d read through heaps of the other kind" % (P["rank"], d))
        ns = ~sw
        Cn, tn = C[ns], t[ns]
        if (src[ns] != Cn).any():
            raise SimError("rank %d dir %d: a source without a transposition is not the child" % (P["rank"], d))
        own = tier_of[Cn] >= 0
        if (tier_of[Cn[own]] != tn[own] - 1).any():
            raise SimError("rank %d dir %d: an own child not in the tier below" % (P["rank"], d))
        rest, j = Cn[~own], tn[~own] // P["batch"]
        ok = np.isin((j << 28) | rest, rk)
        if d < 4:
            ok |= np.isin((j << 28) | ((1 + d) << 20) | rest, rk)
        if not ok.all():
            i = np.nonzero(~ok)[0][0]
            raise SimError("rank %d dir %d: child %#x neither own, filled nor in message %d" % (P["rank"], d, rest[i],
                                                                                          j[i]))
        if received is not None:
            received.update(zip(rest.tolist(), [d] * len(rest)))
    return True


def simulate(P, seed=0):
    """Run all ranks' RCCL-mode op lists (plans built with loopback=0) in one random interleaving."""
    rng = random.Random(seed)
    G = len(P)
    final = [np.zeros(1 << 20, bool) for _ in range(G)]
    mine = [np.zeros(1 << 20, bool) for _ in range(G)]
    for r, p in enumerate(P):
        mine[r][p["boxes"]] = True
    have = [np.zeros((5, 1 << 20), bool) for _ in range(G)]   # [code][box] unpacked (code 0 whole box)
    reads = []
    for p in P:
        rd = []
        for d in range(8):
            idx, C, src, sw, q, pp = direction_reads(p, d)
            rd.append((idx, C, src))
        reads.append(rd)
    tier_boxes = []
    for p in P:
        off = p["off"]
        tier_boxes.append([p["boxes"][off[t]:off[t + 1]] for t in range(len(off) - 1)])
    streams = {}
    bound = {}
    for r, p in enumerate(P):
        last = {}
        for i, (kind, axis, ev, on_x, arg, peer) in enumerate(p["ops"].tolist()):
            streams.setdefault((r, axis) if on_x else (r, "S"), deque()).append(i)
            # one completion event per rank and batch, shared by the axes (dist_box.hip: slot 0)
            if kind == BOP_RECORD:
                last[(ev, arg)] = (r, i)
            elif kind == BOP_WAIT:
                if peer != r:
                    raise SimError("RCCL mode waits on another rank's event")
                if (ev, arg) not in last:
                    raise SimError("rank %d waits on batch %d's event before any record of it" % (r, arg))
                bound[(r, i)] = last[(ev, arg)]
    p2p = {}
    cnt = defaultdict(int)
    for r, p in enumerate(P):
        for i, (kind, axis, ev, on_x, arg, peer) in enumerate(p["ops"].tolist()):
            if kind in (BOP_SEND, BOP_RECV):
                key = ("s", axis, r, peer) if kind == BOP_SEND else ("r", axis, peer, r)
                p2p[(r, i)] = cnt[key]
                cnt[key] += 1
    for (kind, a, s, d), n in list(cnt.items()):
        if kind == "s" and cnt[("r", a, s, d)] != n:
            raise SimError("axis %d: %d sends %d->%d, %d receives" % (a, n, s, d, cnt[("r", a, s, d)]))
    packed = [dict() for _ in range(G)]         # (axis, batch) -> entries
    arrived = [dict() for _ in range(G)]
    done = set()

    def op(r, i):
        return P[r]["ops"][i].tolist()

    def ready(r, i):
        kind, axis, ev, on_x, arg, peer = op(r, i)
        if kind == BOP_WAIT:
            b = bound[(r, i)]
            return b is None or b in done
        if kind in (BOP_SEND, BOP_RECV):
            other = BOP_RECV if kind == BOP_SEND else BOP_SEND
            for key, q in streams.items():
                if key[0] != peer or not q:
                    continue
                o = op(peer, q[0])
                if o[0] == other and o[1] == axis and o[5] == r and p2p[(peer, q[0])] == p2p[(r, i)]:
                    return (peer, q[0])
            return False
        return True

    def execute(r, i):
        p = P[r]
        kind, axis, ev, on_x, arg, peer = op(r, i)
        if kind == BOP_TIER:
            own = tier_boxes[r][arg]
            lo, hi = p["off"][arg], p["off"][arg + 1]
            for d in range(8):
                idx, C, src = reads[r][d]
                k = (idx >= lo) & (idx < hi)
                Ck, sk = C[k], src[k]
                local = (sk != Ck) | mine[r][Ck]
                if not final[r][sk[local]].all():
                    raise SimError("rank %d tier %d: a source of direction %d not computed yet" % (r, arg, d))
                far = Ck[~local]
                ok = have[r][0][far] | (have[r][1 + d][far] if d < 4 else False)
                if not np.all(ok):
                    raise SimError("rank %d tier %d: child %#x not arrived" % (r, arg, far[~ok][0]))
            if final[r][own].any():
                raise SimError("rank %d computes a box twice" % r)
            final[r][own] = True
        elif kind == BOP_PACK:
            raise SimError("rank %d: a pack op (the tier kernel writes the messages)" % r)
        elif kind == BOP_SEND:
            ent = seg(p["send"][axis], arg)
            if not final[r][ent & 0xFFFFF].all():
                raise SimError("rank %d sends message %d on axis %d before its boxes are computed" % (r, arg, axis))
            packed[r][(axis, arg)] = ent.copy()
        elif kind == BOP_RECV:
            ent = packed[peer].get((axis, arg))
            if ent is None:
                raise SimError("rank %d receives message %d that rank %d has not packed" % (r, arg, peer))
            if not np.array_equal(ent, seg(p["recv"][axis], arg)):
                raise SimError("axis %d message %d: rank %d expects other entries than rank %d sends" %
                               (axis, arg, r, peer))
            arrived[r][(axis, arg)] = ent
            if p["direct"]:   # no unpack: the boxes are in the table once the flag is seen
                have[r][ent >> 20, ent & 0xFFFFF] = True
        elif kind == BOP_UNPACK:
            # one launch for every message of the batch
            for a in range(3):
                if not len(seg(p["recv"][a], arg)):
                    continue
                ent = arrived[r].get((a, arg))
                if ent is None:
                    raise SimError("rank %d unpacks message %d on axis %d before it arrived" % (r, arg, a))
                have[r][ent >> 20, ent & 0xFFFFF] = True
        done.add((r, i))

    remaining = sum(len(q) for q in streams.values())
    while remaining:
        cands = []
        for key, q in streams.items():
            if q:
                res = ready(key[0], q[0])
                if res:
                    cands.append((key, res))
        if not cands:
            raise SimError("deadlock; stream heads: %s" % {k: op(k[0], q[0]) for k, q in streams.items() if q})
        key, res = rng.choice(cands)
        r, i = key[0], streams[key].popleft()
        remaining -= 1
        if res is True:
            execute(r, i)
        else:
            pr, pj = res
            pkey = next(k for k, q in streams.items() if k[0] == pr and q and q[0] == pj)
            streams[pkey].popleft()
            remaining -= 1
            pair = sorted([(r, i), (pr, pj)], key=lambda x: op(*x)[0] != BOP_SEND)
            for x in pair:
                execute(*x)
    for r, p in enumerate(P):
        if not final[r][p["boxes"]].all():
            raise SimError("rank %d ends with boxes unsolved" % r)
    return True


def oracle_box_codes(oracle, root):
    """{box: 4096 uint8 codes in box order} of the root's region from the C oracle (codes of
    csrc/gm_common.hpp: WIN R -> R + 1, LOSS R -> 255 - R)."""
    keys, recs = oracle.solve(5, (8,), root=root)
    val, rem = recs >> 14, (recs & 0x3FFF).astype(np.int64)
    codes = np.where(val == 0, rem + 1, 255 - rem).astype(np.uint8)
    idx = np.zeros(len(keys), np.int64)
    k = keys.astype(np.int64)
    for i in range(4):
        idx |= ((k >> (4 * i)) & 3) << (4 + 2 * i)
    for j in range(4):
        idx |= ((k >> (16 + 4 * j)) & 1) << j
    boxes = box_of_key(k)
    out = {}
    order = np.argsort(boxes, kind="stable")
    bs, ix, cs = boxes[order], idx[order], codes[order]
    starts = np.r_[0, np.nonzero(np.diff(bs))[0] + 1, len(bs)]
    for s, e in zip(starts[:-1], starts[1:]):
        a = np.zeros(4096, np.uint8)
        a[ix[s:e]] = cs[s:e]
        out[int(bs[s])] = a
    return out


def gloo_rank(rank, world, root, batch, symmetry, split, result):
    """One rank's RCCL-mode op list on the host over gloo; afterwards every box it computed and
    every row it received equals the oracle's."""
    import torch
    import torch.distributed as dist
    import conftest
    p = load_plan(world, rank, root, batch=batch, symmetry=symmetry, split=split)
    ref = oracle_box_codes(conftest.Oracle(), root)
    table = {}
    own_done = set()
    rows_have = defaultdict(set)
    pending = {}
    off = p["off"]
    mine = set(p["boxes"].tolist())
    for kind, axis, ev, on_x, arg, peer in p["ops"].tolist():
        if kind == BOP_TIER:
            for k, b in enumerate(p["boxes"][off[arg]:off[arg + 1]].tolist()):
                idx = off[arg] + k
                c = coords(b)
                for d in range(8):
                    if c[d] < 1:
                        continue
                    C, src = b - unit(d), int(p["srcs"][idx, d])
                    if src != C or C in mine:
                        assert src in own_done, "rank %d: source %#x of %#x not computed" % (rank, src, b)
                    else:
                        need = entry_rows(0 if d >= 4 else (1 + d) << 20)
                        assert set(need.tolist()) <= rows_have[C], "rank %d: rows of %#x missing" % (rank, C)
                table[b] = ref[b].copy()
                own_done.add(b)
        elif kind == BOP_SEND:
            # the message as the tier kernel left it: each entry's rows of its (final) box
            ent = seg(p["send"][axis], arg)
            assert all((e & 0xFFFFF) in own_done for e in ent.tolist()), "rank %d: send before compute" % rank
            msg = np.concatenate([table[e & 0xFFFFF].reshape(256, 16)[entry_rows(e)].ravel() for e in ent.tolist()])
            t = torch.from_numpy(msg)
            pending[("s", axis, arg)] = (dist.isend(t, dst=peer), t)
        elif kind == BOP_RECV:
            ent = seg(p["recv"][axis], arg)
            n = sum(4096 if (e >> 20) == 0 else 2048 for e in ent.tolist())
            t = torch.empty(n, dtype=torch.uint8)
            pending[("r", axis, arg)] = (dist.irecv(t, src=peer), t)
        elif kind == BOP_UNPACK:
            for a in range(3):
                if ("r", a, arg) not in pending:
                    continue
                w, t = pending.pop(("r", a, arg))
                w.wait()
                data, o = t.numpy(), 0
                for e in seg(p["recv"][a], arg).tolist():
                    rows = entry_rows(e)
                    C = e & 0xFFFFF
                    tab = table.setdefault(C, np.zeros(4096, np.uint8)).reshape(256, 16)
                    tab[rows] = data[o:o + 16 * len(rows)].reshape(-1, 16)
                    o += 16 * len(rows)
                    rows_have[C].update(rows.tolist())
    for w, _ in pending.values():
        w.wait()
    own_ok = all(np.array_equal(table[b], ref[b]) for b in p["boxes"].tolist())
    recv_ok = all(np.array_equal(table[C].reshape(256, 16)[sorted(rows)], ref[C].reshape(256, 16)[sorted(rows)])
                  for C, rows in rows_have.items())
    result.update(rank=rank, own_ok=own_ok, recv_ok=recv_ok, own_boxes=len(p["boxes"]),
                  received_boxes=len(rows_have))


def gloo_main(rank, world, port, root, batch, symmetry, split, queue):
    """Process entry of the world-size-N gloo test (tests/test_box_plan.py)."""
    import os
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for q in (here, os.path.dirname(here)):
        if q not in sys.path:
            sys.path.insert(0, q)
    import torch.distributed as dist
    try:
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
        res = {}
        gloo_rank(rank, world, root, batch, symmetry, split, res)
        dist.barrier()
        dist.destroy_process_group()
        queue.put(res)
    except Exception as e:
        queue.put({"rank": rank, "error": repr(e)})
        raise
