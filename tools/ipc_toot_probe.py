#!/usr/bin/env python3
"""Toot-and-Otto W x H solved by N processes sharing one GPU over the sparse IPC transport, with
per-tier progress on stderr (GM_TRACE=1) -- a development aid for the multi-process path.
Like bench.py's side config: `solves` solves with the symmetry reduction on, then (symoff = 1)
one with it off, in the same contexts.

    python tools/ipc_toot_probe.py 6 4 2 [solves] [symoff]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def rank_main(rank, world, phase, params, solves, symoff):
    import ctypes
    import torch.distributed as tdist
    from gamesmanmpi_amd import Context, _lib
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = Context(_lib.GAME_TOOT, params, device=0)
    uid = [None]
    if rank == 0:
        buf = ctypes.create_string_buffer(128)
        _lib.check(_lib.lib().gm_comm_unique_id(buf, 128))
        uid[0] = buf.raw
    tdist.broadcast_object_list(uid, src=0)
    ctx.set_comm(rank, world, uid[0])
    ctx.set_option(_lib.OPT_SPARSE_TRANSPORT, 1)
    out = []
    for i in range(solves + symoff):
        if i == solves:
            ctx.set_option(_lib.OPT_SYMMETRY, 0)
        phase("solve %d" % i)
        n, rec = ctx.solve(ctx.initial())
        d, m = ctx.digest()
        out.append((n, rec, d, m, ctx.stats()["solve_ms"]))
    ctx.close()
    tdist.destroy_process_group()
    return out


def main():
    w, h, n = (int(x) for x in sys.argv[1:4])
    solves = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    symoff = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    os.environ.setdefault("GM_TRACE", "1")
    import socket
    from mp_ranks import run_ranks
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    res = run_ranks(rank_main, n, ((w, h), solves, symoff), timeout=240)
    for i in range(len(res[0])):
        d = sum(r[i][2] for r in res) & ((1 << 64) - 1)
        print({"solve": i, "positions": res[0][i][0], "root": res[0][i][1], "digest": "%#x" % d,
               "digest_positions": sum(r[i][3] for r in res), "solve_ms": [r[i][4] for r in res]}, flush=True)


if __name__ == "__main__":
    main()
