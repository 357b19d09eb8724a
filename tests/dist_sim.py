"""CPU checks of the sharded dense solve's RCCL-mode schedule (test infrastructure).

The plans come from the product itself: ``gm_dist_plan`` (include/gmsolve.h) runs
the host code gm_solve uses to build each rank's block lists and op list
(csrc/dist_sub.hip plan_shape / plan_lists / build_ops) without touching a GPU.

``simulate`` executes every rank's op list under the semantics the RCCL path
relies on -- one FIFO per HIP stream (S, X[axis]), hipStreamWaitEvent binding to
the latest record of that event enqueued before it, and rendezvous matching of
the k-th ncclSend/ncclRecv per (communicator, peer) -- in a random interleaving of
whatever is ready, and tracks which blocks each rank's table holds final values
for.  A tier launch also writes its blocks' extra destinations (GM_PLAN_XDEST:
symmetric-fill images, halo ring slots), as the tier kernel does.  It fails on a
deadlock, on a tier launch whose child blocks are not final in that rank's table,
on a send of a message whose blocks are not all written, on a ring slot written
before its previous message left or received over before it was unpacked, and on
sender / receiver halo lists that disagree.

``gloo_rank`` runs one rank's op list as a host program over torch.distributed
(gloo) -- the same messages, peers and ordering as RCCL mode, with the oracle's
values as the block payloads -- so two real processes exchange the halos.
"""
import random
from collections import defaultdict, deque

import numpy as np

from gamesmanmpi_amd import _lib

OP_TIER, OP_PACK, OP_UNPACK, OP_SEND, OP_RECV, OP_RECORD, OP_WAIT, OP_FILL = range(8)
EV_PACKED, EV_XCH, EV_UNPACKED = range(3)


def load_plan(heaps, world, rank, batch=4, slots=4, symmetry=1, owner=0):
    kw = dict(batch=batch, slots=slots, symmetry=symmetry, owner=owner)
    shape_off, shape = _lib.dist_plan(heaps, world, rank, _lib.PLAN_SHAPE, **kw)
    low, high, ntiers, b, nbatch, nslots, g = (int(v) for v in shape)
    p = {"rank": rank, "low": low, "high": high, "ntiers": ntiers, "batch": b, "nbatch": nbatch,
         "nslots": nslots, "g": g, "halo_range": shape_off.reshape(-1, 2)}
    p["own_off"], p["own"] = _lib.dist_plan(heaps, world, rank, _lib.PLAN_OWN, **kw)
    p["fill_off"], p["fill"] = _lib.dist_plan(heaps, world, rank, _lib.PLAN_FILL, **kw)
    p["send"], p["recv"] = [], []
    for a in range(max(1, g)):
        p["send"].append(_lib.dist_plan(heaps, world, rank, _lib.PLAN_SEND, axis=a, **kw))
        p["recv"].append(_lib.dist_plan(heaps, world, rank, _lib.PLAN_RECV, axis=a, **kw))
    p["ops"] = _lib.dist_plan(heaps, world, rank, _lib.PLAN_OPS, **kw)[1].reshape(-1, 6).astype(np.int64)
    p["xoff"], p["xd"] = _lib.dist_plan(heaps, world, rank, _lib.PLAN_XDEST, **kw)
    return p


def message_of_tier(p):
    """tier -> the batch whose halo message carries it (-1: none)."""
    m = np.full(p["ntiers"], -1, dtype=np.int64)
    for j, (lo, hi) in enumerate(p["halo_range"].tolist()):
        if lo <= hi:
            m[lo:hi + 1] = j
    return m


def tier_writes(p, t):
    """What tier t's launch writes besides its own blocks: (fill pairs, {axis: (batch, blocks, indices)})."""
    pairs = seg(p["fill_off"], p["fill"], t).reshape(-1, 2)
    sends = {}
    j = message_of_tier(p)[t]
    if j >= 0:
        for a in range(p["g"]):
            blocks = seg(*p["send"][a], j)
            if len(blocks):
                k = np.nonzero(tier_of(blocks, p["high"]) == t)[0]
                if len(k):
                    sends[a] = (int(j), blocks[k], k)
    return pairs, sends


def seg(off, data, i):
    if i < 0 or i + 1 >= len(off):
        return data[:0]
    return data[off[i]:off[i + 1]]


def tier_of(blocks, high):
    t = np.zeros(len(blocks), dtype=np.int64)
    for k in range(high):
        t += (blocks.astype(np.int64) >> (4 * k)) & 15
    return t


def child_blocks(blocks, high):
    """Every (parent index, child high part) pair: one high nibble lowered by 1 or 2."""
    b = blocks.astype(np.int64)
    out_p, out_c = [], []
    for k in range(high):
        h = (b >> (4 * k)) & 15
        for s in (1, 2):
            m = h >= s
            out_p.append(np.nonzero(m)[0])
            out_c.append(b[m] - (s << (4 * k)))
    return np.concatenate(out_p), np.concatenate(out_c)


class SimError(AssertionError):
    pass


def simulate(plans, seed=0):
    """Run all ranks' RCCL-mode op lists in one random interleaving; raise SimError on a violation."""
    rng = random.Random(seed)
    G = len(plans)
    high, ns = plans[0]["high"], plans[0]["nslots"]
    nblocks = 1 << (4 * high)
    final = [np.zeros(nblocks, dtype=bool) for _ in range(G)]
    # streams: (rank, "S") and (rank, axis); each a deque of op indices
    streams = {}
    bound = {}        # (rank, op index) of a WAIT -> (rank, op index) of the RECORD it waits for, or None
    for r, p in enumerate(plans):
        last_record = {}
        for i, (kind, axis, ev, on_x, arg, peer) in enumerate(p["ops"].tolist()):
            key = (r, axis) if on_x else (r, "S")
            streams.setdefault(key, deque()).append(i)
            if kind == OP_RECORD:
                last_record[(ev, axis, arg % ns)] = (r, i)
            elif kind == OP_WAIT:
                if peer != r:
                    raise SimError("RCCL mode waits on another rank's event (rank %d op %d)" % (r, i))
                bound[(r, i)] = last_record.get((ev, axis, arg % ns))
    done = set()
    send_slot = [defaultdict(lambda: None) for _ in range(G)]   # (axis, slot) -> [batch, sent]
    recv_slot = [defaultdict(lambda: None) for _ in range(G)]   # (axis, slot) -> [batch, unpacked]

    def op(r, i):
        return plans[r]["ops"][i].tolist()

    def ready(r, i):
        kind, axis, ev, on_x, arg, peer = op(r, i)
        if kind == OP_WAIT:
            b = bound[(r, i)]
            return b is None or b in done
        if kind in (OP_SEND, OP_RECV):
            # a p2p op completes only together with its match, which must be at the head of its stream
            other = OP_RECV if kind == OP_SEND else OP_SEND
            k = p2p_index[(r, i)]
            for key, q in streams.items():
                if key[0] != peer or not q:
                    continue
                j = q[0]
                o = op(peer, j)
                if o[0] == other and o[1] == axis and o[5] == r and p2p_index[(peer, j)] == k:
                    return (peer, j)
            return False
        return True

    # k-th send from src to dst on an axis matches the k-th recv at dst from src
    p2p_index = {}
    counters = defaultdict(int)
    for r, p in enumerate(plans):
        for i, (kind, axis, ev, on_x, arg, peer) in enumerate(p["ops"].tolist()):
            if kind == OP_SEND:
                p2p_index[(r, i)] = counters[("s", axis, r, peer)]
                counters[("s", axis, r, peer)] += 1
            elif kind == OP_RECV:
                p2p_index[(r, i)] = counters[("r", axis, peer, r)]
                counters[("r", axis, peer, r)] += 1
    for key in set(k[1:] for k in counters):
        a, s, d = key
        if counters[("s", a, s, d)] != counters[("r", a, s, d)]:
            raise SimError("axis %d: %d sends %d->%d but %d receives" % (a, counters[("s", a, s, d)], s, d,
                                                                          counters[("r", a, s, d)]))

    def execute(r, i):
        p = plans[r]
        kind, axis, ev, on_x, arg, peer = op(r, i)
        if kind == OP_TIER:
            own = seg(p["own_off"], p["own"], arg)
            if len(own):
                if (tier_of(own, high) != arg).any():
                    raise SimError("rank %d tier %d lists a block of another tier" % (r, arg))
                pi, ch = child_blocks(own, high)
                bad = ~final[r][ch]
                if bad.any():
                    raise SimError("rank %d tier %d: child block %x of %x not final" %
                                   (r, arg, int(ch[bad][0]), int(own[pi[bad][0]])))
                if final[r][own].any():
                    raise SimError("rank %d computes block %x twice" % (r, int(own[final[r][own]][0])))
                final[r][own] = True
            pairs, sends = tier_writes(p, arg)
            if not final[r][pairs[:, 1]].all():
                raise SimError("rank %d tier %d fills from a block it did not compute" % (r, arg))
            final[r][pairs[:, 0]] = True
            for a, (j, blocks, _) in sends.items():
                prev = send_slot[r][(a, j % ns)]
                if prev is not None and prev[0] != j and not prev[1]:
                    raise SimError("rank %d writes batch %d into the send slot of batch %d before it was sent"
                                   % (r, j, prev[0]))
                if prev is None or prev[0] != j:
                    send_slot[r][(a, j % ns)] = [j, False, set()]
                send_slot[r][(a, j % ns)][2].update(blocks.tolist())
        elif kind == OP_SEND:
            cur = send_slot[r][(axis, arg % ns)]
            if cur is None or cur[0] != arg:
                raise SimError("rank %d sends batch %d from a slot holding %s" % (r, arg, cur and cur[:2]))
            if cur[2] != set(seg(*p["send"][axis], arg).tolist()):
                raise SimError("rank %d sends batch %d on axis %d before all its blocks are written" % (r, arg, axis))
            cur[1] = True
        elif kind == OP_RECV:
            prev = recv_slot[r][(axis, arg % ns)]
            if prev is not None and not prev[1]:
                raise SimError("rank %d receives batch %d over unpacked batch %d" % (r, arg, prev[0]))
            sender = plans[peer]
            got = send_slot[peer][(axis, arg % ns)]
            if got is None or got[0] != arg:
                raise SimError("rank %d receives batch %d but rank %d's slot holds %s" % (r, arg, peer, got and got[:2]))
            mine, theirs = seg(*p["recv"][axis], arg), seg(*sender["send"][axis], arg)
            if not np.array_equal(mine, theirs):
                raise SimError("axis %d batch %d: rank %d expects other blocks than rank %d sends" %
                               (axis, arg, r, peer))
            if not final[peer][theirs].all():
                raise SimError("rank %d's halo of batch %d left non-final" % (peer, arg))
            recv_slot[r][(axis, arg % ns)] = [arg, False]
        elif kind == OP_UNPACK:
            cur = recv_slot[r][(axis, arg % ns)]
            if cur is None or cur[0] != arg:
                raise SimError("rank %d unpacks batch %d from a slot holding %s" % (r, arg, cur))
            cur[1] = True
            final[r][seg(*p["recv"][axis], arg)] = True
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
            stuck = {k: op(k[0], q[0]) for k, q in streams.items() if q}
            raise SimError("deadlock; stream heads: %s" % stuck)
        key, res = rng.choice(cands)
        r, i = key[0], streams[key].popleft()
        remaining -= 1
        if res is True:
            execute(r, i)
        else:                          # rendezvous: the matched pair completes together, send side first
            pr, pj = res
            pkey = next(k for k, q in streams.items() if k[0] == pr and q and q[0] == pj)
            streams[pkey].popleft()
            remaining -= 1
            pair = [(r, i), (pr, pj)]
            pair.sort(key=lambda x: op(*x)[0] != OP_SEND)
            for x in pair:
                execute(*x)
    owned = np.zeros(nblocks, dtype=np.int64)
    for p in plans:
        owned[p["own"]] += 1
    if not (owned == 1).all():
        raise SimError("blocks owned %d..%d times, not exactly once" % (owned.min(), owned.max()))
    for r, p in enumerate(plans):
        if not final[r][p["own"]].all():
            raise SimError("rank %d ends with own blocks unsolved" % r)
    return True


def gloo_rank(rank, world, heaps, batch, slots, symmetry, oracle_codes, result, owner=0):
    """One rank of the RCCL-mode op list executed on the host over torch.distributed
    (gloo): halos travel as real messages; a tier launch copies the oracle's codes for
    its own blocks after checking their child blocks arrived."""
    import torch
    import torch.distributed as dist
    p = load_plan(heaps, world, rank, batch, slots, symmetry, owner)
    low, high, ns = p["low"], p["high"], p["nslots"]
    bsz = 1 << (4 * low)
    table = np.zeros(1 << (4 * heaps), dtype=np.uint8)
    have = np.zeros(1 << (4 * high), dtype=bool)
    sendbuf, recvbuf, pending = {}, {}, {}
    for kind, axis, ev, on_x, arg, peer in p["ops"].tolist():
        if kind == OP_TIER:
            own = seg(p["own_off"], p["own"], arg)
            if len(own):
                _, ch = child_blocks(own, high)
                assert have[ch].all(), "rank %d tier %d: child blocks missing" % (rank, arg)
                for H in own.tolist():
                    table[H * bsz:(H + 1) * bsz] = oracle_codes[H * bsz:(H + 1) * bsz]
                have[own] = True
            # the tier kernel's extra destinations: fill images, halo ring slots
            pairs, sends = tier_writes(p, arg)
            for dst, src in pairs.tolist():
                assert have[src]
                table[dst * bsz:(dst + 1) * bsz] = table[src * bsz:(src + 1) * bsz]
                have[dst] = True
            for a, (j, blocks, idx) in sends.items():
                n = len(seg(*p["send"][a], j))
                key = (a, j % ns)
                if key not in sendbuf or sendbuf[key][0] != j:
                    assert ("s", a, j - ns) not in pending, "ring slot reused before its send left"
                    sendbuf[key] = (j, np.zeros(n * bsz, dtype=np.uint8))
                for H, k in zip(blocks.tolist(), idx.tolist()):
                    sendbuf[key][1][k * bsz:(k + 1) * bsz] = table[H * bsz:(H + 1) * bsz]
        elif kind == OP_SEND:
            j, data = sendbuf[(axis, arg % ns)]
            assert j == arg
            buf = torch.from_numpy(data.copy())
            pending[("s", axis, arg)] = (dist.isend(buf, dst=peer), buf)
        elif kind == OP_RECV:
            n = len(seg(*p["recv"][axis], arg)) * bsz
            buf = torch.empty(n, dtype=torch.uint8)
            recvbuf[(axis, arg % ns)] = buf
            pending[("r", axis, arg)] = (dist.irecv(buf, src=peer), buf)
        elif kind == OP_UNPACK:
            pending.pop(("r", axis, arg))[0].wait()
            data = recvbuf[(axis, arg % ns)].numpy()
            for k, H in enumerate(seg(*p["recv"][axis], arg).tolist()):
                table[H * bsz:(H + 1) * bsz] = data[k * bsz:(k + 1) * bsz]
            have[seg(*p["recv"][axis], arg)] = True
        elif kind == OP_WAIT and ev == EV_XCH and not on_x and ("s", axis, arg) in pending:
            pending.pop(("s", axis, arg))[0].wait()     # ring slot reuse: the send has left
    for w, _ in pending.values():
        w.wait()
    own = p["own"]
    # every byte of every own block and every halo block this rank holds equals the oracle's
    idx = (own.astype(np.int64)[:, None] * bsz + np.arange(bsz)[None, :]).ravel()
    held = np.nonzero(have)[0]
    hidx = (held[:, None] * bsz + np.arange(bsz)[None, :]).ravel()
    result.update(rank=rank, own_ok=bool(np.array_equal(table[idx], oracle_codes[idx])),
                  held_ok=bool(np.array_equal(table[hidx], oracle_codes[hidx])),
                  own_blocks=len(own), halo_blocks=int(have.sum()) - len(own))


def oracle_codes(heaps):
    """The C oracle's table of the subtraction game as 1-byte codes (WIN R -> R+1,
    LOSS R -> 255-R; gm_common.hpp), the payload gloo_rank moves."""
    import conftest
    recs = conftest.Oracle().subtract_dense(heaps)
    val, rem = recs >> 14, (recs & 0x3FFF).astype(np.int64)
    return np.where(val == 0, rem + 1, 255 - rem).astype(np.uint8)


def gloo_main(rank, world, port, heaps, batch, slots, symmetry, queue, owner=0):
    """Process entry of the world-size-N gloo test (tests/test_dist_plan.py)."""
    import os
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.dirname(here)):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    try:
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
        res = {}
        gloo_rank(rank, world, heaps, batch, slots, symmetry, oracle_codes(heaps), res, owner)
        dist.barrier()
        dist.destroy_process_group()
        queue.put(res)
    except Exception as e:          # report instead of hanging the parent
        queue.put({"rank": rank, "error": repr(e)})
        raise
