#!/usr/bin/env python3
"""bench.py -- headline benchmark: strong solve of the 2^32-position subtraction game.

Workload (BASELINE.json config 5): 8 heaps x 4 bits, root 0xFFFFFFFF,
all 2^32 positions reachable.  One step = one complete strong solve (value and
remoteness of every position) by libgmsolve.so's dense tiered kernel; the table
lives in HBM (a torch-allocated uint8 tensor of 1-byte codes adopted by the
library) before the
timed region starts.  Synthetic by construction: the game is the input.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Prints ONE JSON line on rank 0 (driver contract), including
  roofline      bound "hbm": achieved = the tier kernel's COMPULSORY bytes per
                launch (1 B written + 2 producer-tier reads = 3 B per
                position, x positions per launch) / its average launch time from
                HIP events on the launch stream; frac = achieved / 8 TB/s;
                traffic = rocprofv3 PMC HBM-side bytes per launch (profiles/), with
                traffic_frac beside it; the SURVEY edge model (15.5 B/position) is
                kept only as a diagnostic field, it is not an HBM bound for a
                kernel that serves 6 of 14.5 child edges from LDS;
  parity        the solved 2^32 table's gm_digest (all ranks summed) against the C
                oracle's digest of the same table -- live from the cpu_baseline
                leg at N = 1, and the committed oracle value
                (tests/golden/oracle_digests.json) at every N;
  cpu_baseline  the C oracle's dense solver (oracle/gm_oracle.c), OpenMP over
                the host threads the box gives the process, on the full 2^32
                workload (a 7-heap sample if the full one would exceed ~30 s);
  other_configs config 3 (Toot-and-Otto 6x4) and config 4 (Othello 4x4) on the
                sparse engine, hash-sharded over the same N ranks when N > 1,
                each with its oracle digest check and (rank 0, N = 1) a CPU
                baseline from the C oracle's sorted-layer OpenMP solver
                (reported beside the headline, not the metric).
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# The sharded solve drives a compute stream and one exchange stream per split heap
# (3 at 8 GPUs) beside torch's streams; with HIP's default of 4 hardware queues some
# share a queue, and a blocked RCCL receive then holds back the kernels queued behind
# it.  Read by HIP at initialisation, so set before torch is imported.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
EDGE_MODEL_BYTES_PER_POSITION = 15.5  # SURVEY §8d edge model, 1-B records: 1 write + 14.5 child reads (diagnostic)
COMPULSORY_BYTES_PER_POSITION = 3.0  # SURVEY §8d compulsory bound with 1-B records: 1 write + 2 producer-tier reads
ORACLE_DIGESTS = os.path.join(REPO, "tests", "golden", "oracle_digests.json")
METRIC = "positions solved/sec (node) at 1/2/4/8 MI355X; achieved HBM GB/s vs peak"
COLL_DEV = "cuda"   # device of the tensors bench.py's own collectives use ("cpu" under gloo)


def _oracle():
    """ctypes view of the C oracle (test infrastructure: the checker and the CPU baseline)."""
    path = os.path.join(REPO, "oracle", "_build", "liboracle.so")
    if not os.path.exists(path):
        return None
    L = ctypes.CDLL(path)
    P = ctypes.POINTER
    L.oracle_subtract_dense_mt.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    L.oracle_dense_digest.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, P(ctypes.c_uint64)]
    L.oracle_dense_digest_blocks.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                             ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, P(ctypes.c_uint64),
                                             P(ctypes.c_uint64)]
    L.oracle_initial.argtypes = [ctypes.c_int, P(ctypes.c_int32), ctypes.c_int, P(ctypes.c_uint64)]
    L.oracle_solve_layered.argtypes = [ctypes.c_int, P(ctypes.c_int32), ctypes.c_int, ctypes.c_uint64,
                                       ctypes.c_int, P(ctypes.c_uint64), P(ctypes.c_uint64),
                                       P(ctypes.c_uint16), P(ctypes.c_uint64), ctypes.c_int, P(ctypes.c_int)]
    return L


def _cpu_name():
    import platform
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), cpu)
    except OSError:
        pass
    return cpu


THREAD_NOTE = ("threads = OMP_NUM_THREADS, the host-CPU share the box grants one GPU (nproc counts the "
               "whole machine)")


def cpu_baseline(heaps=8):
    """The C oracle's dense solver on the host cores (positions/s), plus the oracle
    digest of the table it built (the headline's live parity check).

    OpenMP over every thread the box gives the process (OMP_NUM_THREADS), in the
    GPU's block/tier decomposition (oracle/gm_oracle.c oracle_subtract_dense_mt).
    The full 8-heap workload takes ~4 s on 16 cores; if a 7-heap probe says it
    would exceed ~30 s, the 7-heap sample is reported instead."""
    L = _oracle()
    if L is None:
        return None, None
    import numpy as np
    threads = L.oracle_threads()

    def run(h):
        out = np.empty(1 << (4 * h), dtype=np.uint16)
        t0 = time.perf_counter()
        rc = L.oracle_subtract_dense_mt(h, out.ctypes.data, 0)
        dt = time.perf_counter() - t0
        return (dt if rc == 0 else None), out

    dt, _ = run(heaps - 1)
    if dt is None:
        return None, None
    digest = None
    if dt * 16 < 30.0:
        dt8, out = run(heaps)
        if dt8 is not None:
            d = ctypes.c_uint64()
            L.oracle_dense_digest(out.ctypes.data, ctypes.c_uint64(len(out)), 0, ctypes.byref(d))
            digest = d.value
            dt = dt8
        else:
            heaps -= 1
        del out
    else:
        heaps -= 1
    n = 1 << (4 * heaps)
    return ({"value": n / dt, "unit": "positions/s", "cores": threads, "kind": "port",
             "sample": "%d-heap subtraction game, all %d positions, %.2f s; C oracle dense retrograde "
                       "(oracle/gm_oracle.c oracle_subtract_dense_mt), OpenMP %d threads on %s; %s, nproc %d"
                       % (heaps, n, dt, threads, _cpu_name(), THREAD_NOTE, os.cpu_count())},
            digest if heaps == 8 else None)


def sparse_cpu_baseline(game, params, root=None, what=None):
    """C oracle's sorted-layer OpenMP solver (oracle_solve_layered) on the host cores:
    positions/s of one complete strong solve of `game` at `params` from `root`
    (default: the initial position)."""
    L = _oracle()
    if L is None:
        return None
    arr = (ctypes.c_int32 * len(params))(*params)
    if root is None:
        r = ctypes.c_uint64()
        L.oracle_initial(game, arr, len(params), ctypes.byref(r))
        root = r.value
    npos, dg, rr, nt = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint16(), ctypes.c_int()
    t0 = time.perf_counter()
    rc = L.oracle_solve_layered(game, arr, len(params), ctypes.c_uint64(root), 0, ctypes.byref(npos),
                                ctypes.byref(dg), ctypes.byref(rr), None, 0, ctypes.byref(nt))
    dt = time.perf_counter() - t0
    if rc != 0:
        return None
    return {"value": npos.value / dt, "unit": "positions/s", "cores": L.oracle_threads(), "kind": "port",
            "positions": npos.value, "seconds": dt, "digest": dg.value, "root_record": rr.value,
            "sample": "%s %s, %s: all %d positions, %.2f s; C oracle sorted-layer retrograde "
                      "(oracle/gm_oracle.c oracle_solve_layered), OpenMP %d threads on %s; %s"
                      % ({3: "Toot-and-Otto", 4: "Othello"}[game], "x".join(map(str, params)),
                         what or "from the initial position", npos.value, dt, L.oracle_threads(), _cpu_name(),
                         THREAD_NOTE)}


def committed_digest(name):
    """Oracle digest of a full table from tests/golden/oracle_digests.json (made by
    tests/golden/make_oracle_digests.py with the C oracle), or None."""
    try:
        with open(ORACLE_DIGESTS) as f:
            return json.load(f).get(name)
    except (OSError, ValueError):
        return None


def summed_digest(ctx, world, dist, torch):
    """gm_digest of this rank's table, summed over ranks (mod 2^64) when world > 1."""
    d, m = ctx.digest()
    if world > 1:
        v = torch.tensor([d - (1 << 64) if d >= (1 << 63) else d, m], dtype=torch.int64, device=COLL_DEV)
        dist.all_reduce(v)
        d, m = int(v[0].item()) & ((1 << 64) - 1), int(v[1].item())
    return d, m


def rank_digest_check(heaps, world, root, rank_digests, batch, slots, symmetry, owner):
    """N > 1: each rank's gm_digest covers exactly its own blocks (csrc/dist_sub.hip
    dist_sub_digest); compare every one with the C oracle's digest over the same
    blocks (the rank's GM_PLAN_OWN list, host-only plan of the same options), so a
    rank whose part of the table is wrong is named.  Rank 0 only; ~5 s of host work."""
    L = _oracle()
    if L is None:
        return None
    import numpy as np
    from gamesmanmpi_amd import _lib
    rec = np.empty(1 << (4 * heaps), dtype=np.uint16)
    if L.oracle_subtract_dense_mt(heaps, rec.ctypes.data, 0) != 0:
        return None
    low = int(_lib.dist_plan(heaps, world, 0, _lib.PLAN_SHAPE, batch=batch, slots=slots, symmetry=symmetry,
                             owner=owner)[1][0])
    out = []
    for r in range(world):
        own = np.ascontiguousarray(_lib.dist_plan(heaps, world, r, _lib.PLAN_OWN, batch=batch, slots=slots,
                                                  symmetry=symmetry, owner=owner)[1], dtype=np.uint32)
        d, c = ctypes.c_uint64(), ctypes.c_uint64()
        L.oracle_dense_digest_blocks(rec.ctypes.data, heaps, low, ctypes.c_uint64(root), own.ctypes.data,
                                     ctypes.c_uint64(len(own)), 0, ctypes.byref(d), ctypes.byref(c))
        got_d, got_n = rank_digests[r]
        out.append({"rank": r, "blocks": int(len(own)), "positions": got_n,
                    "ok": (got_d, got_n) == (d.value, c.value)})
    return {"ranks": out, "wrong_ranks": [x["rank"] for x in out if not x["ok"]]}


def box_sharding(world, args, root, st, rstats, per_rank, autotune, torch, dist):
    """The sharding block of the split box engine (csrc/dist_box.hip): the
    plan's boxes per rank -- one work set divided, work_vs_one_gpu = the boxes all ranks
    compute / the boxes one GPU computes = 1 -- and the halo bytes each rank received."""
    from gamesmanmpi_amd import _lib
    G = world if world > 1 else args.virtual_ranks
    kw = dict(batch=args.dist_batch, symmetry=args.dist_symmetry)
    boxes = [int(_lib.box_plan(G, r, _lib.BOXPLAN_COUNTS, root, **kw)[0]) for r in range(G)]
    one = int(_lib.box_plan(1, 0, _lib.BOXPLAN_COUNTS, root, **kw)[0]) if G > 1 else sum(boxes)
    sh = _lib.box_plan(G, 0, _lib.BOXPLAN_SHAPE, root, **kw).astype(int).tolist()
    axes = ["heap %d box coordinate >= %d" % (sh[8 + 4 * a], sh[9 + 4 * a]) for a in range(sh[1])]
    recv = rstats[0]["recv_bytes"] if (world > 1 and rstats) else None
    if world > 1:
        t = torch.tensor([float(st["exchanged_bytes"]), float(recv or 0)], dtype=torch.float64, device=COLL_DEV)
        allr = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allr, t)
        sent = [int(a[0].item()) for a in allr]
        recvd = [int(a[1].item()) for a in allr]
    else:
        sent, recvd = [st["exchanged_bytes"]], [r["recv_bytes"] for r in rstats]
    return {
        "scheme": ("box engine split: the 2^20 boxes of the 4x4x4x4x2x2x2x2 lattice divided by halves of %d heap "
                   "coordinate(s) (%s); ranks >= 2^%d idle; each box computed by exactly one rank; a child box "
                   "of the other half read through a same-kind heap transposition of an own box (symmetric "
                   "fill) or received: %s (DESIGN.md §5.0)"
                   % (sh[1], "; ".join(axes), sh[1],
                      ("the lower rank's tier kernel writes it to a message slot and an exchange stream per axis "
                       "sends each batch of %d tiers over RCCL" % args.dist_batch)
                      if (world > 1 and args.box_transport != "ipc") else
                      ("the lower rank's tier kernel stores it straight into the receiver's table, one signal "
                       "per batch of %d tiers" % args.dist_batch))),
        "work_vs_one_gpu": sum(boxes) / max(1, one),
        "boxes_per_rank": boxes,
        "halo_batch_tiers": args.dist_batch, "halo_batch_autotune_ms": autotune,
        "halo_symmetric_fill": bool(args.dist_symmetry),
        "halo_transport": ("direct stores into the peer's table mapped through HIP IPC, device flags "
                           "(GM_OPT_BOX_TRANSPORT 1)"
                           if args.box_transport == "ipc" else "RCCL send / recv, one communicator per axis")
                          if world > 1 else "loopback (direct stores between the virtual ranks' tables, event per batch)",
        "halo_transport_verified_before_this_run": ("IPC: across 2-4 processes sharing ONE GPU, with poisoned halos "
                                                    "and an injected early-read fault (tests/test_gpu_multiproc.py); "
                                                    "RCCL: the op lists over gloo on the CPU only; neither between "
                                                    "two GPUs (no multi-GPU box in the build pipeline) -- this run's "
                                                    "probe and per-rank oracle digests are the check"
                                                    if world > 1 else None),
        "halo_bytes_sent_per_step_by_rank": sent,
        "halo_bytes_received_per_step_by_rank": recvd,
        "per_rank_gpu_ms_and_enqueue_ms_per_step": per_rank,
        "round4_note": ("round 4's N>1 numbers (1.86/3.29/5.17x at 2/4/8 on one GPU's clock) came from each "
                        "rank computing one member per heap-permutation orbit -- a symmetry reduction of the "
                        "work, not a division of one work set; this split computes every box once")}


def box_rank_digest_check(world, root, rank_digests):
    """N > 1, box engine: each rank's gm_digest covers exactly the boxes it owns
    (csrc/dense_box.hip, gm_box_plan GM_BOXPLAN_OWN); compare every one with the C
    oracle's digest over the same boxes (oracle_dense_digest_boxes), so a rank whose part
    of the table is wrong is named.  Rank 0 only; ~10 s of host work."""
    L = _oracle()
    if L is None:
        return None
    import numpy as np
    from gamesmanmpi_amd import _lib
    L.oracle_dense_digest_boxes.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                            ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                                            ctypes.POINTER(ctypes.c_uint64)]
    rec = np.empty(1 << 32, dtype=np.uint16)
    if L.oracle_subtract_dense_mt(8, rec.ctypes.data, 0) != 0:
        return None
    out = []
    for r in range(world):
        own = np.ascontiguousarray(_lib.box_plan(world, r, _lib.BOXPLAN_OWN, root), dtype=np.uint32)
        d, c = ctypes.c_uint64(), ctypes.c_uint64()
        L.oracle_dense_digest_boxes(rec.ctypes.data, ctypes.c_uint64(root), own.ctypes.data,
                                    ctypes.c_uint64(len(own)), 0, ctypes.byref(d), ctypes.byref(c))
        got_d, got_n = rank_digests[r]
        out.append({"rank": r, "boxes_owned": int(len(own)), "positions": got_n,
                    "ok": (got_d, got_n) == (d.value, c.value)})
    return {"ranks": out, "wrong_ranks": [x["rank"] for x in out if not x["ok"]]}


TOOT_6X4_PER_PLY = [1, 12, 114, 748, 4266, 19692, 81140, 285708, 928196, 2665424, 7098172, 17010952,
                    37792450, 64636776, 100084356, 136321692, 169785424, 180777508, 172831136,
                    135153280, 91440950, 45953432, 19196602, 4537828, 606968]


SIDE_WARMUP, SIDE_REPEATS = 1, 5   # median of 5 runs after 1 warm-up
# --rehearse-one-gpu: the side configs' ranks share device 0 and exchange over the sparse
# engine's IPC transport (RCCL refuses two ranks on one GPU)
SIDE_DEVICE, SIDE_SPARSE_IPC = None, False


def toot_sample_root(params=(6, 4), plies=3):
    """The bounded CPU sample of config 3: the Toot-and-Otto 6x4 position after `plies`
    moves, taking at ply i the child (n // 2 + i) % n of the n children in gen_moves
    order (csrc/games.hpp host twin, gm_expand_host).  After 3 plies the subgame has
    106.4 M positions: ~7 s for the C oracle on the box's 16 host threads (after 4
    plies 46.8 M, 3.3 s)."""
    from gamesmanmpi_amd import games
    hd = games.HostDescriptor(games.TootCodec(*params))
    k = hd.initial()
    try:
        for i in range(plies):
            kids = hd.expand(k)[1]
            k = kids[(len(kids) // 2 + i) % len(kids)]
    finally:
        hd.close()
    return k


def timed_solves(ctx, root, rank, world, dist, torch, warmup=SIDE_WARMUP, repeats=SIDE_REPEATS):
    """Solve times (s, max over ranks) of `repeats` solves after `warmup` untimed ones."""
    for _ in range(warmup):
        ctx.solve(root)
    ts = []
    for _ in range(repeats):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n, rec = ctx.solve(root)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64, device=COLL_DEV)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        ts.append(dt)
    return n, rec, ts


def sparse_config(name, game, params, rank, world, dist, torch):
    """Config 3 / 4 on the sparse engine, hash-sharded over the job's ranks (RCCL p2p,
    csrc/dist_sparse.hip) when world > 1.  Checked: position count, root record,
    per-ply counts (Toot 6x4: SURVEY Appendix D) and the full-table digest summed
    over ranks against the C oracle's (tests/golden/oracle_digests.json).  Time =
    max over ranks, median of 5 after 1 warm-up."""
    from gamesmanmpi_amd import Context, _lib
    ctx = Context(game, params, device=SIDE_DEVICE if SIDE_DEVICE is not None else int(os.environ.get("LOCAL_RANK", 0)))
    if world > 1:
        uid = [None]
        if rank == 0:
            buf = ctypes.create_string_buffer(128)
            _lib.check(_lib.lib().gm_comm_unique_id(buf, 128))
            uid[0] = buf.raw
        dist.broadcast_object_list(uid, src=0)
        ctx.set_comm(rank, world, uid[0])
        if SIDE_SPARSE_IPC:
            ctx.set_option(_lib.OPT_SPARSE_TRANSPORT, 1)
    root = ctx.initial()
    n, rec, ts = timed_solves(ctx, root, rank, world, dist, torch)
    med = sorted(ts)[len(ts) // 2]
    st = ctx.stats()
    # positions counted vs computed: with GM_OPT_SYMMETRY on (the default)
    # the engine expands and resolves one representative per symmetry orbit and counts every
    # position of the orbit; both rates are reported
    out = {"positions": n, "root_record": rec, "solve_ms": med * 1e3, "positions_per_s": n / med,
           "positions_computed": st["n_stored"], "positions_computed_per_s": st["n_stored"] / med,
           "positions_note": "positions = every position reached (each symmetry orbit counted whole); "
                             "positions_computed = the orbit representatives the engine expanded and resolved "
                             "(GM_OPT_SYMMETRY 1, the default)",
           "statistic": "median of %d solves after %d warm-up (max over ranks)" % (SIDE_REPEATS, SIDE_WARMUP),
           "solve_ms_all": [round(t * 1e3, 3) for t in ts],
           "ranks": world, "exchanged_bytes_rank%d" % rank: st["exchanged_bytes"],
           "transport": None if world == 1 else ("IPC, the ranks sharing one GPU (rehearsal)" if SIDE_SPARSE_IPC
                                                 else "RCCL, one GPU per rank")}
    ref = committed_digest(name)
    d, m = summed_digest(ctx, world, dist, torch)
    out["digest"] = "%#018x" % d
    out["digest_matches_oracle"] = (ref is not None and (d, m) == (ref["digest"], ref["positions"])
                                    and rec == ref["root_record"])
    if name == "toot_6x4":
        out["workload"] = "Toot-and-Otto 6x4 (config 3), sparse engine" + (", hash-sharded" if world > 1 else "")
        out["per_ply_counts_match_appendix_d"] = [int(x) for x in ctx.tier_counts()] == TOOT_6X4_PER_PLY
        out["ok"] = n == 1187212827 and out["per_ply_counts_match_appendix_d"] and out["digest_matches_oracle"]
        out["edges"] = st["n_edges"]
        out["algo_bytes_per_position"] = st["algo_bytes"] / n
        if world == 1:
            out["roofline"] = toot_roofline(st["algo_bytes"], med)
        # the same solve with the symmetry reduction off: every position computed
        ctx.set_option(_lib.OPT_SYMMETRY, 0)
        fn, frec, fts = timed_solves(ctx, root, rank, world, dist, torch, warmup=1, repeats=3)
        fmed = sorted(fts)[1]
        fst = ctx.stats()
        fd, fm = summed_digest(ctx, world, dist, torch)
        out["symmetry_off"] = {"solve_ms": fmed * 1e3, "positions": fn, "positions_computed": fst["n_stored"],
                               "positions_per_s": fn / fmed, "edges": fst["n_edges"],
                               "statistic": "median of 3 after 1 warm-up (max over ranks)",
                               "digest": "%#018x" % fd,
                               "digest_matches_oracle": (ref is not None and (fd, fm) == (ref["digest"], ref["positions"])
                                                         and frec == ref["root_record"])}
        ctx.set_option(_lib.OPT_SYMMETRY, 1)
        if world == 1:   # the CPU leg's bounded sample, solved here too: the same workload on both
            sub = toot_sample_root(params)
            sn, srec, sts = timed_solves(ctx, sub, rank, world, dist, torch, warmup=1, repeats=3)
            sm = sorted(sts)[1]
            out["sample_on_gpu"] = {"root": "%#x" % sub, "positions": sn, "root_record": srec,
                                    "solve_ms": sm * 1e3, "positions_per_s": sn / sm,
                                    "statistic": "median of 3 after 1 warm-up"}
    else:
        out["workload"] = "Othello 4x4 (config 4), sparse engine" + (", hash-sharded" if world > 1 else "")
        out["ok"] = n == 54089 and (rec >> 14) == 1 and (rec & 0x3FFF) == 12 and out["digest_matches_oracle"]
    ctx.close()
    return out


# Othello at the reference's default 8x8 board (othello_bit_new.py:8) on the device, 128-bit keys
# (DESIGN.md §4.4): positions of the seed-5 playout from the standard start with E empty squares
# (tools/othello8_scale.py playout_roots; E = 10 is tests/plugins/othello8_endgame.py's root,
# pinned by the reference plugin's golden table in tests/test_gpu_othello8.py)
OTHELLO8_ROOTS = {10: "303800204018057a4646bfdebfe6fa800200", 14: "30300c2c503841784646b1d2afc6be000200",
                  16: "3030242050384178460699daafc6be000200", 18: "30302420583e4160460699daa7c0bc100200"}
OTHELLO8_EMPTIES = int(os.environ.get("GM_BENCH_OTHELLO8_EMPTIES", 16))


def othello8_config(rank, world, dist, torch):
    """§8f.3 on the device: one seed-5 endgame of OTHELLO8_EMPTIES empty squares, one GPU
    (rank 0 at N = 1 only).  Parity: the same root on 8 virtual ranks gives the same digest,
    position count and root record (the 10-empty root is pinned to the reference plugin's
    golden table by tests/test_gpu_othello8.py).  Time: median of 3 solves after 1 warm-up."""
    from gamesmanmpi_amd import Context, _lib, games
    e = OTHELLO8_EMPTIES
    codec = games.OthelloCodec(8, 8)
    key = codec.key(bytes.fromhex(OTHELLO8_ROOTS[e]).decode("latin-1"))
    ctx = Context(_lib.GAME_OTHELLO, (8, 8), device=int(os.environ.get("LOCAL_RANK", 0)))
    n, rec, ts = timed_solves(ctx, key, rank, 1, dist, torch, warmup=1, repeats=3)
    med = sorted(ts)[1]
    st = ctx.stats()
    d1 = ctx.digest()
    ctx.close()
    v = Context(_lib.GAME_OTHELLO, (8, 8), device=int(os.environ.get("LOCAL_RANK", 0)))
    v.set_option(_lib.OPT_VIRTUAL_RANKS, 8)
    vn, vrec = v.solve(key)
    d8 = v.digest()
    v.close()
    return {"workload": "Othello 8x8 (the reference plugin's default board), seed-5 playout position with %d "
                        "empty squares, 128-bit keys, sparse engine on one GPU" % e,
            "root_hex": OTHELLO8_ROOTS[e], "positions": n, "root_record": rec, "solve_ms": med * 1e3,
            "solve_ms_all": [round(t * 1e3, 3) for t in ts], "positions_per_s": n / med,
            "statistic": "median of 3 solves after 1 warm-up", "edges": st["n_edges"], "tiers": st["n_tiers"],
            "table_gb": st["table_bytes"] / 1e9, "digest": "%#018x" % d1[0],
            "roofline": (sparse_roofline(None, med, OTHELLO8_PROFILE, ("self_expand_kernel", "self_retro_kernel"),
                                         "kernel_sum_ms_per_replay") if e == 16 else None),
            "ok": (vn, vrec, d8) == (n, rec, d1),
            "parity": "the same root on 8 virtual ranks (hash-sharded, loopback exchange): digest, positions and "
                      "root record equal"}


RANDOM_LOAD_PEAK = 47e9   # random 16-B loads/s from an 8 GiB table (tools/randbench.hip, profiles/r01_randbench.txt)
RANDOM_CAS_PEAK = 17e9    # random 8-B CAS/s from an 8 GiB table (same)
TOOT_PROFILE = os.path.join(REPO, "profiles", "traffic_toot6x4.json")


def toot_roofline(algo_bytes, solve_s):
    """Config 3's roofline.  The sparse engine is bound by the random-
    access rate, not by bytes: every insert and lookup moves a 64-B line.
    So the block grades the two kernels that make 80 % of a solve, expand (one probe per edge,
    a CAS per new key) and retro (one lookup per undecided child), by their memory-side
    request rates from the committed profile (profiles/traffic_toot6x4.json: rocprofv3
    kernel trace of replayed solves + one-solve PMC passes, tools/sparse_replay_profile.py)
    against the measured random-access peaks; and it sets the counted HBM-side bytes of a
    solve beside the SURVEY §8d algorithmic bytes (10 + 18 d per position)."""
    return sparse_roofline(algo_bytes, solve_s, TOOT_PROFILE, ("expand_kernel", "retro_kernel"),
                           "kernel_sum_ms_per_replay")


def sparse_roofline(algo_bytes, solve_s, path, names, sum_key):
    try:
        prof = json.load(open(path))
    except (OSError, ValueError):
        return None
    ks = prof["kernels"]
    per = {}
    for k in names:
        x = ks[k]
        sec = x["ms"] / 1e3
        per[k] = {"ms": x["ms"], "ea_read_req": x["ea_read_req"], "ea_write_req": x["ea_write_req"],
                  "read_req_per_s": x["ea_read_req"] / sec, "write_req_per_s": x["ea_write_req"] / sec,
                  "frac_of_random_load_peak": x["ea_read_req"] / sec / RANDOM_LOAD_PEAK,
                  "requests_per_s": (x["ea_read_req"] + x["ea_write_req"]) / sec,
                  "l2_hit": x["l2_hit"]}
    rd = sum(per[k]["ea_read_req"] for k in per)
    wr = sum(per[k]["ea_write_req"] for k in per)
    sec = sum(per[k]["ms"] for k in per) / 1e3
    counted = sum(x["fetch_bytes"] + x["write_bytes"] for x in ks.values())
    return {"bound": "random access", "unit": "requests/s",
            "achieved": rd / sec, "peak": RANDOM_LOAD_PEAK, "frac": rd / sec / RANDOM_LOAD_PEAK,
            "frac_all_requests": (rd + wr) / sec / RANDOM_LOAD_PEAK,
            "achieved_note": "memory-side read requests of the two kernels per second of their kernel time "
                             "(requests_per_s per kernel adds the write requests: CAS and stores)",
            "peak_cas_per_s": RANDOM_CAS_PEAK,
            "peak_source": "tools/randbench.hip (profiles/r01_randbench.txt): random 16-B loads 47 G/s, "
                           "random 8-B CAS 17 G/s, 8 GiB table",
            "kernels": per,
            "algo_bytes_per_solve": algo_bytes, "algo_gbs": algo_bytes / solve_s / 1e9 if algo_bytes else None,
            "algo_frac_of_hbm_peak": algo_bytes / solve_s / 1e9 / HBM_PEAK_GBS if algo_bytes else None,
            "counted_bytes_per_solve": counted, "counted_over_algo_bytes": counted / algo_bytes if algo_bytes else None,
            "profile": os.path.relpath(path, REPO),
            "profile_kernel_sum_ms": min(prof[sum_key])}


OTHELLO8_PROFILE = os.path.join(REPO, "profiles", "traffic_othello8_16.json")


SPARSE_CPU_SAMPLE = {"othello_4x4": (4, (4, 4)),    # the whole config-4 workload
                     "toot_6x4": (3, (6, 4))}        # bounded sample: the 6x4 board from a ply-4 position


def other_configs(rank, world, dist, torch, budget_s=240.0, emit=None):
    """Run the side configs under a watchdog: if the ranks have not finished within
    budget_s (a sharded exchange that never completes), every rank prints what it
    has (rank 0 the headline line via emit) and leaves with status 0, so the
    headline measurement is never lost to a side measurement."""
    import threading
    from gamesmanmpi_amd import _lib
    res = {}

    def expire():
        res["error"] = "watchdog: side configs did not finish within %.0f s" % budget_s
        if emit is not None:
            emit(res)
        sys.stdout.flush()
        os._exit(0)

    timer = threading.Timer(budget_s, expire)
    timer.daemon = True
    timer.start()
    for name, game, params in (("othello_4x4", _lib.GAME_OTHELLO, (4, 4)), ("toot_6x4", _lib.GAME_TOOT, (6, 4))):
        try:
            res[name] = sparse_config(name, game, params, rank, world, dist, torch)
        except Exception as e:  # reported in the line; a rank that fails here leaves the others to the watchdog
            res[name] = {"error": "%s: %s" % (type(e).__name__, e)}
            if world > 1:
                break
        if rank == 0 and world == 1 and "error" not in res[name]:
            g, p = SPARSE_CPU_SAMPLE[name]
            if name == "toot_6x4":
                smp = res[name]["sample_on_gpu"]
                cb = sparse_cpu_baseline(g, p, root=int(smp["root"], 16),
                                         what="the subgame of the position %s after 3 plies (toot_sample_root)"
                                              % smp["root"])
                if cb is not None:
                    cb["matches_gpu_sample"] = (cb["positions"] == smp["positions"]
                                                and cb["root_record"] == smp["root_record"])
                    res[name]["speedup_vs_cpu_baseline_same_sample"] = smp["positions_per_s"] / cb["value"]
            else:
                cb = sparse_cpu_baseline(g, p)
            if cb is not None:
                res[name]["cpu_baseline"] = cb
                res[name]["speedup_vs_cpu_baseline"] = res[name]["positions_per_s"] / cb["value"]
    if world == 1 and rank == 0 and not os.environ.get("GM_BENCH_NO_OTHELLO8"):
        try:
            res["othello_8x8_endgame"] = othello8_config(rank, world, dist, torch)
        except Exception as e:  # reported in the line
            res["othello_8x8_endgame"] = {"error": "%s: %s" % (type(e).__name__, e)}
    timer.cancel()
    return res


def pmc_traffic(heaps):
    """HBM bytes per launch / per solve of the tier kernel from a committed rocprofv3 PMC summary."""
    path = os.path.join(REPO, "profiles", "traffic_subtract%d.json" % heaps)
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        t = json.load(f)
    return t.get("hbm_bytes_per_launch"), t.get("hbm_bytes_per_solve")


def copy_bandwidth(torch, nbytes=1 << 31, reps=10):
    """Measured device-to-device copy bandwidth (read + write bytes / s), SURVEY §8d."""
    a = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    gbs = 2.0 * nbytes * reps / (e0.elapsed_time(e1) / 1e3) / 1e9
    del a, b
    return gbs


def main():
    if os.environ.get("GM_BENCH_STACKS"):   # development: every rank's Python stacks on stderr after N s
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["GM_BENCH_STACKS"]), repeat=True)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--heaps", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-toot", action="store_true", help="skip the config-3/4 side measurements")
    ap.add_argument("--cpu-heaps", type=int, default=8)
    ap.add_argument("--dist-batch", type=int, default=None,
                    help="N>1: tiers per halo exchange (default: chosen in warmup by the max-over-ranks solve "
                         "time, from 1, 2, 4 on the box engine and 1, 2, 4, 8 on the block engine; %d for "
                         "virtual ranks)" % 1)
    ap.add_argument("--dist-slots", type=int, default=4, help="N>1: halo buffers per split heap")
    ap.add_argument("--dist-symmetry", type=int, default=1, choices=(0, 1),
                    help="N>1: fill halo blocks that are a heap permutation of an own block locally")
    ap.add_argument("--dist-owner", type=int, default=0, choices=(0, 1),
                    help="N>1: block owner, 0 = split heaps in halves (default), 1 = tier-balanced (measured "
                         "slower per rank on one GPU, DESIGN.md §5)")
    ap.add_argument("--block-engine", action="store_true",
                    help="8 heaps: run the block engine (GM_OPT_SUB_INTERLEAVE 10) instead of the box engine, "
                         "sharded with halo exchanges at N > 1 (the round-3 multi-GPU path, for comparison)")
    ap.add_argument("--box-transport", choices=("rccl", "ipc"), default="ipc",
                    help="N>1, 8 heaps: the tier kernel stores halo boxes straight into the peer's table mapped "
                         "through HIP IPC, over xGMI, and each rank's solve replays as one captured graph "
                         "(GM_OPT_BOX_TRANSPORT 1, default: one node; also runs with several ranks on one GPU), or "
                         "halo messages over RCCL send / recv, launched eagerly (the library's default transport)")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="N>1 rehearsal on a one-GPU box: every rank on device 0, bench.py's collectives over "
                         "gloo, the box engine's halos and the side configs' exchanges over the IPC transports "
                         "(RCCL refuses two ranks on one GPU); the ranks share the GPU, so the times are not "
                         "multi-GPU results")
    ap.add_argument("--virtual-ranks", type=int, default=1,
                    help="diagnostic: run the sharded algorithm with V loopback ranks on this one GPU")
    ap.add_argument("--watchdog", type=float, default=None,
                    help="seconds before the headline solve is declared hung (default 240 + 2 s per step)")
    args = ap.parse_args()
    if args.dist_owner == 1 and not args.dist_symmetry:
        ap.error("--dist-owner 1 needs --dist-symmetry 1 (the tier-balanced owner relies on the symmetric fill)")

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    global COLL_DEV, SIDE_DEVICE, SIDE_SPARSE_IPC
    if args.rehearse_one_gpu:
        if args.heaps != 8 or args.block_engine:
            ap.error("--rehearse-one-gpu runs the 8-heap box engine")
        local, COLL_DEV, args.box_transport = 0, "cpu", "ipc"
        SIDE_DEVICE, SIDE_SPARSE_IPC = 0, True
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE %d" % (args.gpus, world))

    # Headline watchdog: a sharded solve whose exchange never completes must end the
    # job with a non-zero status (never a re-exec), not hang until the driver's limit.
    import threading
    budget = args.watchdog or (240.0 + 2.0 * (args.steps + args.warmup))

    def expire():
        sys.stderr.write("bench.py rank %d: watchdog: the headline solve did not finish within %.0f s\n"
                         % (rank, budget))
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": None, "error": "watchdog expired after %.0f s" % budget}),
                  flush=True)
        sys.stderr.flush()
        os._exit(3)

    watchdog = threading.Timer(budget, expire)
    watchdog.daemon = True
    watchdog.start()

    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    if world > 1:
        if args.rehearse_one_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from gamesmanmpi_amd import Context, _lib

    ctx = Context(_lib.GAME_SUBTRACT, (args.heaps,), device=local)
    # the box engine (csrc/dense_box.hip) at 8 heaps: one GPU, and at N > 1 the boxes split
    # over the ranks by halves of heap coordinates, halo boxes stored into the receiving rank's
    # table (IPC transport) or exchanged over the library's RCCL communicators per batch of
    # tiers (csrc/dist_box.hip); else the block engine
    box = args.heaps == 8 and not args.block_engine
    if not box:
        ctx.set_option(_lib.OPT_SUB_INTERLEAVE, 10)
    if box and args.box_transport == "ipc":
        ctx.set_option(_lib.OPT_BOX_TRANSPORT, 1)
    if world > 1:
        uid = [None]
        if rank == 0:
            buf = ctypes.create_string_buffer(128)
            _lib.check(_lib.lib().gm_comm_unique_id(buf, 128))
            uid[0] = buf.raw
        dist.broadcast_object_list(uid, src=0)
        ctx.set_comm(rank, world, uid[0])
    # Every rank keeps the table in the global key layout (it writes only its own
    # blocks and the halo it receives), so each GPU holds 1 B x 16^heaps.
    table = torch.empty(1 << (4 * args.heaps), dtype=torch.uint8, device="cuda")
    ctx.adopt_dense_table(table.data_ptr(), table.numel())
    # A dedicated (non-null) stream: the tier launches are replayed as a hipGraph,
    # which cannot be captured on the legacy default stream.
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    ctx.set_option(_lib.OPT_TIMING, 1)
    default_batch = 1 if box else 4   # box: B = 1 modelled fastest at 2, 4, 8 ranks (profiles/r05d_box_split_time.txt)
    ctx.set_option(_lib.OPT_DIST_BATCH, args.dist_batch or default_batch)
    ctx.set_option(_lib.OPT_DIST_SLOTS, args.dist_slots)
    ctx.set_option(_lib.OPT_DIST_SYMMETRY, args.dist_symmetry)
    ctx.set_option(_lib.OPT_DIST_OWNER, args.dist_owner)
    if args.virtual_ranks > 1:
        ctx.set_option(_lib.OPT_VIRTUAL_RANKS, args.virtual_ranks)
    root = ctx.initial()

    def barrier():
        if world > 1:
            dist.barrier()

    transport_fallback = None
    if world > 1 and box and args.box_transport == "ipc":
        # untimed probe: the IPC transport's cross-process schedule has run on hardware with the
        # ranks sharing one GPU only.  If a probe solve fails on any rank, or the summed digest
        # is not the committed oracle digest, every rank falls back to RCCL together.  Received
        # boxes are poisoned (GM_OPT_POISON 1): every rank's table starts as 0xFF, and each
        # halo box goes back to 0xFF once read, so solve 2 reads nothing solve 1 left -- a halo
        # that lands late, or is read from a stale line, changes that solve's digest
        # (tests/test_gpu_multiproc.py::test_box_ipc_early_read_caught_by_poison injects one).
        err = ""
        ref = committed_digest("subtract_%d" % args.heaps) if root == (1 << (4 * args.heaps)) - 1 else None
        bad = 0.0
        ctx.set_option(_lib.OPT_POISON, 1)
        for k in range(2):
            try:
                ctx.solve(root)
            except _lib.GMError as e:
                err = str(e)
            if os.environ.get("GM_BENCH_PROBE_FAIL") == "1":   # test hook: report a failed probe
                err = err or "probe failure forced (GM_BENCH_PROBE_FAIL)"
            flag0 = torch.tensor([1.0 if err else 0.0], dtype=torch.float64, device=COLL_DEV)
            dist.all_reduce(flag0, op=dist.ReduceOp.MAX)   # every rank makes the same collectives
            if flag0.item() > 0:
                bad = 1.0
                break
            if ref is not None:
                d, nd = summed_digest(ctx, world, dist, torch)   # the same sum on every rank
                if (d, nd) != (ref["digest"], ref["positions"]):
                    bad, err = 1.0, "solve %d: summed digest %#x differs from the committed oracle digest" % (k + 1, d)
                    break
        ctx.set_option(_lib.OPT_POISON, 0)   # the timed solves run the plain schedule
        flag = torch.tensor([bad], dtype=torch.float64, device=COLL_DEV)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        if flag.item() > 0:
            msgs = [None] * world
            dist.all_gather_object(msgs, err)
            transport_fallback = "IPC transport probe failed (%s)" % "; ".join(
                "rank %d: %s" % (r, m) for r, m in enumerate(msgs) if m)
            if not args.rehearse_one_gpu:   # (ranks sharing one GPU: RCCL refuses, nothing to fall back to)
                transport_fallback += "; halos over RCCL instead"
                args.box_transport = "rccl"
                ctx.set_option(_lib.OPT_BOX_TRANSPORT, 0)
            sys.stderr.write("bench.py rank %d: %s\n" % (rank, transport_fallback))
            barrier()
            if args.rehearse_one_gpu:   # nothing to fall back to: one clean non-zero exit
                if rank == 0:
                    print(json.dumps({"metric": METRIC, "value": None, "error": transport_fallback}), flush=True)
                watchdog.cancel()
                ctx.close()
                dist.destroy_process_group()
                sys.exit(4)

    autotune = None
    if world > 1 and args.dist_batch is None:
        # untimed: the halo batch trades the upper ranks' lag (B - 1 tiers) against the
        # number of RCCL messages; every rank measures the same candidates and takes
        # the same argmin of the max-over-ranks time, so all ranks keep one schedule
        autotune = {}
        for b in ((1, 2, 4) if box else (1, 2, 4, 8)):
            ctx.set_option(_lib.OPT_DIST_BATCH, b)
            ctx.solve(root)
            barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                ctx.solve(root)
            torch.cuda.synchronize()
            dt = torch.tensor([(time.perf_counter() - t0) / 3 * 1e3], dtype=torch.float64, device=COLL_DEV)
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
            autotune["batch%d" % b] = (round(float(dt.item()), 4), b)
        _, args.dist_batch = min(autotune.values())
        autotune = {k: v[0] for k, v in autotune.items()}
        ctx.set_option(_lib.OPT_DIST_BATCH, args.dist_batch)
    args.dist_batch = args.dist_batch or default_batch
    for _ in range(args.warmup):
        n, rec = ctx.solve(root)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kernel_ms = 0.0
    enqueue_ms = 0.0
    launches = 0
    for _ in range(args.steps):
        n, rec = ctx.solve(root)
        st = ctx.stats()
        kernel_ms += st["kernel_ms"]
        launches += st["kernel_launches"]
        enqueue_ms += st["forward_ms"] if (world > 1 or args.virtual_ranks > 1) else 0.0
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    per_rank = None
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=COLL_DEV)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # each rank's own view per step: GPU time of its sharded solve (HIP events on its
        # stream, halo waits included) and host time spent enqueueing it
        mine = torch.tensor([kernel_ms / args.steps, enqueue_ms / args.steps], dtype=torch.float64, device=COLL_DEV)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = [[round(float(x), 4) for x in a.tolist()] for a in allr]

    # parity of the last timed solve: the whole table's digest (summed over ranks)
    # against the C oracle's digest of the same table
    digest, ndig = summed_digest(ctx, world, dist, torch)
    rank_parity = None
    if world > 1:
        d0, m0 = ctx.digest()
        mine = torch.tensor([d0 - (1 << 64) if d0 >= (1 << 63) else d0, m0], dtype=torch.int64, device=COLL_DEV)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        if rank == 0 and args.virtual_ranks == 1:
            got = [(int(a[0].item()) & ((1 << 64) - 1), int(a[1].item())) for a in allr]
            rank_parity = (box_rank_digest_check(world, root, got) if box else
                           rank_digest_check(args.heaps, world, root, got, args.dist_batch, args.dist_slots,
                                             args.dist_symmetry, args.dist_owner))
        barrier()
    watchdog.cancel()
    g = 0
    for i in range(args.heaps):
        g ^= ((root >> (4 * i)) & 15) % 3
    closed_form_ok = (rec >> 14) == (1 if g == 0 else 0)   # LOSS iff xor over heaps of (h mod 3) == 0
    ref = committed_digest("subtract_%d" % args.heaps) if root == (1 << (4 * args.heaps)) - 1 else None
    parity = {"digest": "%#018x" % digest, "positions_in_digest": ndig, "root_record": rec,
              "root_closed_form_ok": closed_form_ok,
              "matches_committed_oracle_digest": (None if ref is None else
                                                  (digest, ndig, rec) == (ref["digest"], ref["positions"],
                                                                          ref["root_record"])),
              "matches_live_oracle_digest": None,
              "per_rank_vs_oracle": rank_parity}

    positions = n
    value = positions * args.steps / elapsed
    st = ctx.stats()
    launches_per_solve = max(1, launches // max(1, args.steps))
    traffic_launch, traffic_solve = pmc_traffic(args.heaps)
    copy_gbs = copy_bandwidth(torch) if world == 1 else None
    kernel_s_per_solve = kernel_ms / 1e3 / max(1, args.steps)
    avg_launch_s = (kernel_ms / 1e3) / max(1, launches)
    # algorithmic (compulsory) bytes per launch: 3 B x the positions this rank's launches solve
    # (box engine at N > 1: its boxes, tie boxes included -- they are computed here too)
    rstats = ctx.rank_stats() if box else []
    own_positions = positions if world == 1 else positions / world
    if box and (world > 1 or args.virtual_ranks > 1) and rstats:
        # the launches timed here are this process's: one rank's at N > 1, every virtual
        # rank's (run one after another on this GPU) with --virtual-ranks
        own_positions = sum(r["boxes"] for r in rstats) * 4096.0
    sharded = world > 1 or args.virtual_ranks > 1
    if sharded:
        # the committed PMC summary is of the one-GPU solve's launches, not of a rank's
        traffic_launch, traffic_solve = None, None
    compulsory_per_launch = COMPULSORY_BYTES_PER_POSITION * own_positions / launches_per_solve
    achieved = compulsory_per_launch / avg_launch_s / 1e9 if avg_launch_s > 0 else None
    traffic_gbs = (traffic_launch / avg_launch_s / 1e9) if (traffic_launch and avg_launch_s > 0) else None
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "positions/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (the game itself: every position of the 2^32-state subtraction game)",
        "config": {"workload": "subtraction game, %d heaps x 4 bits, root %#x (config 5)" % (args.heaps, root),
                   "positions": positions,
                   "parallelism": "1 GPU" if world == 1 else ("box-split x%d" if box else "block-sharded x%d")
                   % world},
        "parity": parity,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                     "traffic": traffic_launch,
                     "traffic_gbs": traffic_gbs,
                     "traffic_frac": (traffic_gbs / HBM_PEAK_GBS) if traffic_gbs else None,
                     "kernel": (("box_tier_kernel<%s> (csrc/dense_box.hip: 4x4x4x4x2x2x2x2 boxes, one launch "
                                 "per box-tier%s)" % (("true", "; this rank's boxes, its halo message slots written "
                                                       "by the same kernel") if sharded else ("false", ""))
                                 if launches_per_solve > max(1, args.virtual_ranks) else
                                 "box_flow_kernel<%s> (csrc/dense_box.hip: 4x4x4x4x2x2x2x2 boxes, every box-tier in "
                                 "one launch, a box group starting when its child boxes are stored%s)"
                                 % ("false", ""))
                                if box else
                                "sub_tier_kernel_wk<%d> (tiers of >= 4096 blocks), sub_tier_kernel_b4<%d> (smaller)"
                                % (args.heaps - 3, args.heaps - 3)),
                     "algo_bytes_per_position": COMPULSORY_BYTES_PER_POSITION,
                     "algo_bytes_model": "compulsory: 1 B code written + 2 B producer-tier reads per position",
                     "launches_per_solve": launches_per_solve,
                     "avg_launch_us": avg_launch_s * 1e6,
                     "kernel_ms_per_solve": kernel_ms / max(1, args.steps),
                     "traffic_bytes_per_position": (traffic_solve / positions) if traffic_solve else None,
                     "traffic_source": "profiles/traffic_subtract%d.json (rocprofv3 --pmc FETCH_SIZE x2 + "
                                       "WRITE_SIZE, per launch)" % args.heaps,
                     "diag_survey_edge_model_bytes_per_position": 2 * EDGE_MODEL_BYTES_PER_POSITION,
                     "diag_survey_edge_model_gbs": (2 * EDGE_MODEL_BYTES_PER_POSITION * own_positions
                                                    / kernel_s_per_solve / 1e9 if kernel_s_per_solve > 0 else None),
                     "diag_survey_edge_model_note": "SURVEY §8d's graded edge model with u16 records (31 B/position): "
                                                    "above the HBM peak because the box kernel serves child edges from "
                                                    "LDS and registers; compulsory bytes are graded (DESIGN.md §6)",
                     "diag_edge_model_bytes_per_position": EDGE_MODEL_BYTES_PER_POSITION,
                     "diag_edge_model_gbs": (EDGE_MODEL_BYTES_PER_POSITION * own_positions / kernel_s_per_solve / 1e9
                                             if kernel_s_per_solve > 0 else None),
                     "measured_copy_gbs": copy_gbs,
                     "timing": ("HIP events bracketing each solve's tier-launch graph replay on the launch "
                                "stream; avg launch = span / launches (includes in-graph gaps)"
                                if (world == 1 or box) else
                                "HIP events around this rank's whole sharded solve (includes halo waits)")},
        "exchanged_bytes_per_step_rank0": st["exchanged_bytes"],
        "sharding": None if (world == 1 and args.virtual_ranks == 1) else box_sharding(
            world, args, root, st, rstats, per_rank, autotune, torch, dist) if box else {
            "halo_batch_tiers": args.dist_batch, "halo_batch_autotune_ms": autotune, "halo_slots": args.dist_slots,
            "halo_symmetric_fill": bool(args.dist_symmetry),
            "block_owner": ("split heaps in halves", "tier-balanced")[args.dist_owner],
            "host_enqueue_ms_per_step_rank0": enqueue_ms / max(1, args.steps),
            "per_rank_gpu_ms_and_enqueue_ms_per_step": per_rank},
        "cpu_baseline": None,
        "halo_transport_fallback": transport_fallback,
        "rehearsal": ("--rehearse-one-gpu: %d ranks sharing ONE GPU (gloo for bench.py's collectives, IPC transport "
                      "for the halos); not a multi-GPU measurement" % world if args.rehearse_one_gpu else None),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"], live = cpu_baseline(args.cpu_heaps)
        if live is not None and args.heaps == args.cpu_heaps == 8 and root == 0xFFFFFFFF:
            parity["matches_live_oracle_digest"] = live == digest
    parity["ok"] = bool(closed_form_ok and parity["matches_committed_oracle_digest"] is not False
                        and parity["matches_live_oracle_digest"] is not False
                        and not (rank_parity and rank_parity["wrong_ranks"]))
    ctx.close()
    if args.virtual_ranks == 1 and not args.no_toot:
        del table
        torch.cuda.empty_cache()

        def emit(partial):
            if rank == 0:
                out["other_configs"] = partial
                print(json.dumps(out), flush=True)

        out["other_configs"] = other_configs(rank, world, dist, torch, emit=emit)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not parity["ok"]:
        sys.stderr.write("bench.py: PARITY FAILURE of the headline table: %s\n" % json.dumps(parity))
        sys.exit(2)


if __name__ == "__main__":
    try:
        main()
    except SystemExit:
        raise
    except BaseException as e:   # one error line on rank 0 instead of a bare traceback
        import traceback
        traceback.print_exc()
        if int(os.environ.get("RANK", 0)) == 0:
            print(json.dumps({"metric": METRIC, "value": None, "error": "%s: %s" % (type(e).__name__, e)}), flush=True)
        sys.exit(1)
