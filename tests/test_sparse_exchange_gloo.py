"""The hash-sharded sparse engine's RCCL op list replayed over gloo on the CPU (VERDICT r05
item 1's floor; csrc/dist_sparse.hip).

On a one-GPU box the engine's RCCL transport cannot run with two processes (RCCL refuses two
ranks on one device), so its cross-process exchange is replayed here with the library's own
layout (gm_sparse_layout, the function every transport uses) and real data: the reference
plugin's Othello 4x4 golden table.

Forward, per tier t (LOOK_UP, reference src/new_process.py:156-160), each rank
  1. generates its interior positions' children with the descriptor's host twin
     (gm_expand_host) and bins them by (owner = (mix64(key) >> 32) % world, tier step) -- the
     engine's bucket_kernel, which also records each key's parent;
  2. all-gathers the per-bin counts (ncclAllGather) and takes its layout;
  3. sends each owner its segment and receives its own, with the offsets the RCCL branch
     passes to ncclSend / ncclRecv (send_off -> recv_off; one isend / irecv per peer, as one
     ncclGroup), and keeps -- as the owner -- the keys it received, checking each is its own
     and in the tier its bin says (insert_bins_kernel inserts them).
Backward, tiers deepest first (RESOLVE, :179-187): each owner answers the keys it kept for the
tier with their scores from the golden table (lookup_bins_kernel), in the same layout, sends
them back (recv_off -> send_off), and each sender folds them into the parents it recorded
(fold_kernel) and turns the best into the parent's record (finalize_kernel), which must equal
the golden record of the parent.  No key moves in the backward pass.
"""
import os

import numpy as np
import pytest

from conftest import golden

M64 = (1 << 64) - 1
WIN, LOSS, TIE, UNDECIDED = 0, 1, 2, 4
S = 3   # DescOthello::MAX_SKIP


def mix64(x):
    x ^= x >> 33
    x = (x * 0xff51afd7ed558ccd) & M64
    x ^= x >> 33
    x = (x * 0xc4ceb9fe1a85ec53) & M64
    return x ^ (x >> 33)


def owner(k, world):
    return (mix64(k) >> 32) % world


# gm_common.hpp: records <-> preference scores, parent score of the best child
def score_of_record(r):
    v, rem = r >> 14, r & 0x3FFF
    return 0x4000 | rem if v == WIN else (0x8000 | (0x3FFF - rem) if v == TIE else 0xC000 | (0x3FFF - rem))


def parent_score(b):
    low, cls = b & 0x3FFF, b >> 14
    return 0x8000 - low if cls == 3 else (b - 1 if cls == 2 else 0xFFFE - low)


def record_of_score(s):
    cls, low = s >> 14, s & 0x3FFF
    return low if cls == 1 else ((0x8000 | (0x3FFF - low)) if cls == 2 else (0x4000 | (0x3FFF - low)))


def _rank_main(rank, world, phase):
    import torch
    import torch.distributed as dist
    from gamesmanmpi_amd import _lib, games
    dist.init_process_group("gloo", rank=rank, world_size=world)
    keys, recs = golden("othello_4x4")
    table = dict(zip(keys.tolist(), recs.tolist()))
    hd = games.HostDescriptor(games.OthelloCodec(4, 4))
    phase("expand")
    info = {k: hd.expand(k) for k in table}          # key -> (primitive, children, tier)
    hd.close()
    mine = [k for k in table if owner(k, world) == rank]
    tiers = sorted({info[k][2] for k in table})

    def exchange(src, soff, dst, doff):
        reqs = []
        for p in range(world):
            a, b, x, y = int(soff[p]), int(soff[p + 1]), int(doff[p]), int(doff[p + 1])
            if p == rank:
                dst[x:y] = src[a:b]
                continue
            if b > a:
                out = src[a:b].clone()
                reqs.append((dist.isend(out, p), out, None, None))
            if y > x:
                buf = torch.zeros(y - x, dtype=src.dtype)
                reqs.append((dist.irecv(buf, p), buf, x, y))
        for work, buf, x, y in reqs:
            work.wait()
            if x is not None:
                dst[x:y] = buf

    kept = {}   # tier -> (parents, sendp, layout, keys received as the owner)
    checked = sent = 0
    for t in tiers:                                  # forward: LOOK_UP
        phase("forward tier %d" % t)
        parents = [k for k in mine if info[k][2] == t and info[k][0] == UNDECIDED]
        bins = [[] for _ in range(world * S)]
        for i, k in enumerate(parents):
            for c in info[k][1]:
                dt = info[c][2] - t
                assert 1 <= dt <= S
                bins[owner(c, world) * S + dt - 1].append((c, i))
        row = torch.tensor([len(b) for b in bins], dtype=torch.int64)
        allr = [torch.zeros_like(row) for _ in range(world)]
        dist.all_gather(allr, row)
        mat = torch.stack(allr).numpy().astype(np.uint64)
        lay = [a.astype(np.int64) for a in _lib.sparse_layout(world, S, mat, rank)]
        seg, send_off, recv_off, recv_seg = lay
        sendk = torch.zeros(int(send_off[-1]), dtype=torch.int64)
        sendp = np.zeros(int(send_off[-1]), dtype=np.int64)
        for b, lst in enumerate(bins):
            for j, (c, i) in enumerate(lst):
                sendk[seg[b] + j] = c
                sendp[seg[b] + j] = i
        recvk = torch.zeros(int(recv_off[-1]), dtype=torch.int64)
        exchange(sendk, send_off, recvk, recv_off)
        for q in range(world):
            for s in range(S):
                a = int(recv_seg[q * S + s])
                for j in range(a, a + int(mat[q, rank * S + s])):
                    c = int(recvk[j])
                    assert owner(c, world) == rank and info[c][2] == t + 1 + s, "a key reached the wrong rank/tier"
        kept[t] = (parents, sendp, (send_off, recv_off), recvk)
        sent += int(send_off[-1]) - int(send_off[rank + 1] - send_off[rank])
    for t in reversed(tiers):                        # backward: RESOLVE only
        phase("backward tier %d" % t)
        parents, sendp, (send_off, recv_off), recvk = kept.pop(t)
        reply = torch.tensor([score_of_record(table[int(c)]) for c in recvk.tolist()], dtype=torch.int64)
        reply_in = torch.zeros(int(send_off[-1]), dtype=torch.int64)
        exchange(reply, recv_off, reply_in, send_off)
        best = [0] * len(parents)
        for j in range(len(reply_in)):
            best[sendp[j]] = max(best[sendp[j]], int(reply_in[j]))
        for i, k in enumerate(parents):
            assert record_of_score(parent_score(best[i])) == table[k], "parent %#x" % k
            checked += 1
    dist.barrier()
    dist.destroy_process_group()
    return {"rank": rank, "checked": checked, "sent": sent}


def test_layout_restated():
    """gm_sparse_layout equals the layout as include/gmsolve.h states it, on random matrices."""
    from gamesmanmpi_amd import _lib
    rng = np.random.default_rng(5)
    for world, steps in ((1, 1), (2, 3), (3, 2), (8, 3)):
        mat = rng.integers(0, 50, size=(world, world * steps)).astype(np.uint64)
        for r in range(world):
            seg, so, ro, rs = _lib.sparse_layout(world, steps, mat, r)
            row = mat[r].astype(np.int64)
            assert list(seg) == list(np.concatenate([[0], np.cumsum(row)[:-1]]))
            assert list(so) == [int(row[:p * steps].sum()) for p in range(world + 1)]
            col = mat[:, r * steps:(r + 1) * steps].astype(np.int64)
            assert list(ro) == [int(col[:q].sum()) for q in range(world + 1)]
            assert list(rs) == list(np.concatenate([[0], np.cumsum(col.reshape(-1))[:-1]]))


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_replay_of_the_rccl_exchange_othello_4x4(world):
    import socket
    from mp_ranks import run_ranks
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    res = run_ranks(_rank_main, world, (), timeout=240)
    keys, recs = golden("othello_4x4")
    assert sum(r["checked"] for r in res) == int(((recs >> 14) != 3).sum()) - _primitives(keys)
    assert sum(r["sent"] for r in res) > 0


def _primitives(keys):
    from gamesmanmpi_amd import games
    hd = games.HostDescriptor(games.OthelloCodec(4, 4))
    n = sum(1 for k in keys.tolist() if hd.expand(k)[0] != UNDECIDED)
    hd.close()
    return n
