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
  roofline      the tier kernel's algorithmic bytes per launch (SURVEY §8d edge
                model with 1-byte records: 1 + 14.5 = 15.5 B per position, x
                positions per launch) / its average launch time, from
                HIP events recorded around every launch on the launch stream;
                traffic = rocprofv3 PMC bytes per launch from profiles/ when present;
  cpu_baseline  the C oracle's dense solver (oracle/gm_oracle.c), OpenMP over
                the host threads the box gives the process, on the full 2^32
                workload (a 7-heap sample if the full one would exceed ~30 s);
  other_configs config 3 (Toot-and-Otto 6x4) and config 4 (Othello 4x4) on the
                sparse engine, hash-sharded over the same N ranks when N > 1
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

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
ALGO_BYTES_PER_POSITION = 15.5  # SURVEY §8d edge model at 8 heaps, 1-B records: 1 write + 14.5 child reads
COMPULSORY_BYTES_PER_POSITION = 3.0  # SURVEY §8d compulsory bound with 1-B records: 1 write + 2 producer-tier reads
METRIC = "positions solved/sec (node) at 1/2/4/8 MI355X; achieved HBM GB/s vs peak"


def cpu_baseline(heaps=8):
    """The C oracle's dense solver on the host cores (positions/s).

    OpenMP over every thread the box gives the process (OMP_NUM_THREADS), in the
    GPU's block/tier decomposition (oracle/gm_oracle.c oracle_subtract_dense_mt).
    The full 8-heap workload takes ~5-20 s on 16 cores; if a 7-heap probe says it
    would exceed ~30 s, the 7-heap sample is reported instead."""
    path = os.path.join(REPO, "oracle", "_build", "liboracle.so")
    if not os.path.exists(path):
        return None
    import numpy as np
    L = ctypes.CDLL(path)
    L.oracle_subtract_dense_mt.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    threads = L.oracle_threads()

    def run(h):
        out = np.empty(1 << (4 * h), dtype=np.uint16)
        t0 = time.perf_counter()
        rc = L.oracle_subtract_dense_mt(h, out.ctypes.data, 0)
        dt = time.perf_counter() - t0
        return (dt if rc == 0 else None), out

    dt, _ = run(heaps - 1)
    if dt is None:
        return None
    if dt * 16 < 30.0:
        dt8, out = run(heaps)
        if dt8 is not None:
            # spot check against the closed form: LOSS iff xor of (h mod 3) == 0
            k = 0xFFFFFFFF >> (4 * (8 - heaps))
            g = 0
            for i in range(heaps):
                g ^= ((k >> (4 * i)) & 15) % 3
            assert (int(out[k]) >> 14) == (1 if g == 0 else 0)
            dt, heaps = dt8, heaps
        else:
            heaps -= 1
    else:
        heaps -= 1
    n = 1 << (4 * heaps)
    import platform
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), cpu)
    except OSError:
        pass
    return {"value": n / dt, "unit": "positions/s", "cores": threads, "kind": "port",
            "sample": "%d-heap subtraction game, all %d positions, %.2f s; C oracle dense retrograde "
                      "(oracle/gm_oracle.c oracle_subtract_dense_mt), OpenMP %d threads on %s, "
                      "nproc %d" % (heaps, n, dt, threads, cpu, os.cpu_count())}


TOOT_6X4_PER_PLY = [1, 12, 114, 748, 4266, 19692, 81140, 285708, 928196, 2665424, 7098172, 17010952,
                    37792450, 64636776, 100084356, 136321692, 169785424, 180777508, 172831136,
                    135153280, 91440950, 45953432, 19196602, 4537828, 606968]


def sparse_config(name, game, params, rank, world, dist, torch, repeats=2):
    """Config 3 / 4 on the sparse engine, hash-sharded over the job's ranks (RCCL p2p,
    csrc/dist_sparse.hip) when world > 1.  Checked: position count and root record
    (Othello 4x4: SURVEY §8a, 54,089 positions, LOSS in 12; Toot 6x4: Appendix D's
    per-ply counts).  Othello 4x4 at world > 1 also compares the all-reduced
    full-table digest with a one-GPU solve of the same game.  Time = max over ranks."""
    from gamesmanmpi_amd import Context, _lib
    ctx = Context(game, params, device=int(os.environ.get("LOCAL_RANK", 0)))
    if world > 1:
        uid = [None]
        if rank == 0:
            buf = ctypes.create_string_buffer(128)
            _lib.check(_lib.lib().gm_comm_unique_id(buf, 128))
            uid[0] = buf.raw
        dist.broadcast_object_list(uid, src=0)
        ctx.set_comm(rank, world, uid[0])
    root = ctx.initial()
    best = None
    for _ in range(repeats):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n, rec = ctx.solve(root)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64, device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        best = dt if best is None else min(best, dt)
    st = ctx.stats()
    out = {"positions": n, "root_record": rec, "solve_ms": best * 1e3, "positions_per_s": n / best,
           "ranks": world, "exchanged_bytes_rank%d" % rank: st["exchanged_bytes"]}
    if name == "toot_6x4":
        out["workload"] = "Toot-and-Otto 6x4 (config 3), sparse engine" + (", hash-sharded" if world > 1 else "")
        out["per_ply_counts_match_appendix_d"] = [int(x) for x in ctx.tier_counts()] == TOOT_6X4_PER_PLY
        out["ok"] = n == 1187212827 and out["per_ply_counts_match_appendix_d"]
        out["edges"] = st["n_edges"]
        out["algo_bytes_per_position"] = st["algo_bytes"] / n
    else:
        out["workload"] = "Othello 4x4 (config 4), sparse engine" + (", hash-sharded" if world > 1 else "")
        out["ok"] = n == 54089 and (rec >> 14) == 1 and (rec & 0x3FFF) == 12
        if world > 1:
            d, m = ctx.digest()
            v = torch.tensor([d - (1 << 64) if d >= (1 << 63) else d, m], dtype=torch.int64, device="cuda")
            dist.all_reduce(v)
            dsum, msum = int(v[0].item()) & ((1 << 64) - 1), int(v[1].item())
            one = Context(game, params, device=int(os.environ.get("LOCAL_RANK", 0)))
            one.solve(one.initial())
            out["digest_matches_one_gpu"] = (dsum, msum) == one.digest()
            out["ok"] = out["ok"] and out["digest_matches_one_gpu"]
            one.close()
    ctx.close()
    return out


def other_configs(rank, world, dist, torch, budget_s=150.0, emit=None):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--heaps", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-toot", action="store_true", help="skip the config-3/4 side measurements")
    ap.add_argument("--cpu-heaps", type=int, default=8)
    ap.add_argument("--dist-batch", type=int, default=None,
                    help="N>1: tiers per halo exchange (default: chosen in warmup from 1, 2, 4, 8 by the "
                         "max-over-ranks solve time; 4 for virtual ranks)")
    ap.add_argument("--dist-slots", type=int, default=4, help="N>1: halo buffers per split heap")
    ap.add_argument("--dist-symmetry", type=int, default=1, choices=(0, 1),
                    help="N>1: fill halo blocks that are a heap permutation of an own block locally")
    ap.add_argument("--dist-owner", type=int, default=None, choices=(0, 1),
                    help="N>1: block owner, 0 = split heaps in halves, 1 = tier-balanced (default: chosen "
                         "in warmup with the halo batch; 0 for virtual ranks)")
    ap.add_argument("--virtual-ranks", type=int, default=1,
                    help="diagnostic: run the sharded algorithm with V loopback ranks on this one GPU")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE %d" % (args.gpus, world))

    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from gamesmanmpi_amd import Context, _lib

    ctx = Context(_lib.GAME_SUBTRACT, (args.heaps,), device=local)
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
    ctx.set_option(_lib.OPT_DIST_BATCH, args.dist_batch or 4)
    ctx.set_option(_lib.OPT_DIST_SLOTS, args.dist_slots)
    ctx.set_option(_lib.OPT_DIST_SYMMETRY, args.dist_symmetry)
    ctx.set_option(_lib.OPT_DIST_OWNER, args.dist_owner or 0)
    if args.virtual_ranks > 1:
        ctx.set_option(_lib.OPT_VIRTUAL_RANKS, args.virtual_ranks)
    root = ctx.initial()

    def barrier():
        if world > 1:
            dist.barrier()

    autotune = None
    if world > 1 and (args.dist_batch is None or args.dist_owner is None):
        # untimed: the halo batch trades the upper ranks' lag (B - 1 tiers) against the
        # number of RCCL messages, the owner function the ranks' tier balance against
        # the symmetric-fill writes; every rank measures the same candidates and takes
        # the same argmin of the max-over-ranks time, so all ranks keep one schedule
        autotune = {}
        owners = (0, 1) if args.dist_owner is None else (args.dist_owner,)
        batches = (1, 2, 4, 8) if args.dist_batch is None else (args.dist_batch,)
        for o, b in [(o, b) for o in owners for b in batches]:
            if o == 1 and not args.dist_symmetry:
                continue
            ctx.set_option(_lib.OPT_DIST_OWNER, o)
            ctx.set_option(_lib.OPT_DIST_BATCH, b)
            ctx.solve(root)
            barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                ctx.solve(root)
            torch.cuda.synchronize()
            dt = torch.tensor([(time.perf_counter() - t0) / 3 * 1e3], dtype=torch.float64, device="cuda")
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
            autotune["owner%d_batch%d" % (o, b)] = (round(float(dt.item()), 4), o, b)
        _, args.dist_owner, args.dist_batch = min(autotune.values())
        autotune = {k: v[0] for k, v in autotune.items()}
        ctx.set_option(_lib.OPT_DIST_OWNER, args.dist_owner)
        ctx.set_option(_lib.OPT_DIST_BATCH, args.dist_batch)
    args.dist_batch = args.dist_batch or 4
    args.dist_owner = args.dist_owner or 0
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
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # each rank's own view per step: GPU time of its sharded solve (HIP events on its
        # stream, halo waits included) and host time spent enqueueing it
        mine = torch.tensor([kernel_ms / args.steps, enqueue_ms / args.steps], dtype=torch.float64, device="cuda")
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = [[round(float(x), 4) for x in a.tolist()] for a in allr]

    # closed-form check of the root: LOSS iff xor over heaps of (h mod 3) == 0
    g = 0
    for i in range(args.heaps):
        g ^= ((root >> (4 * i)) & 15) % 3
    assert (rec >> 14) == (1 if g == 0 else 0), "root record %#x contradicts the closed form" % rec

    positions = n
    value = positions * args.steps / elapsed
    st = ctx.stats()
    launches_per_solve = max(1, launches // max(1, args.steps))
    traffic_launch, traffic_solve = pmc_traffic(args.heaps)
    copy_gbs = copy_bandwidth(torch) if world == 1 else None
    kernel_s_per_solve = kernel_ms / 1e3 / max(1, args.steps)
    compulsory_gbs = (COMPULSORY_BYTES_PER_POSITION * positions / kernel_s_per_solve / 1e9
                      if kernel_s_per_solve > 0 else None)
    # bytes this rank's tier launches move, per the SURVEY §8d model
    algo_per_launch = st["algo_bytes"] / launches_per_solve
    avg_launch_s = (kernel_ms / 1e3) / max(1, launches)
    achieved = algo_per_launch / avg_launch_s / 1e9 if avg_launch_s > 0 else None
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
                   "positions": positions, "parallelism": "1 GPU" if world == 1 else "block-sharded x%d" % world},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                     "traffic": traffic_launch,
                     "kernel": "sub_tier_kernel_b4<%d>" % (args.heaps - 3),
                     "launches_per_solve": launches_per_solve,
                     "avg_launch_us": avg_launch_s * 1e6,
                     "kernel_ms_per_solve": kernel_ms / max(1, args.steps),
                     "algo_bytes_per_position": ALGO_BYTES_PER_POSITION,
                     "survey_u16_model_bytes_per_position": 31.0,
                     "traffic_bytes_per_position": (traffic_solve / positions) if traffic_solve else None,
                     "traffic_gbs": (traffic_solve / kernel_s_per_solve / 1e9) if traffic_solve else None,
                     "compulsory_bytes_per_position": COMPULSORY_BYTES_PER_POSITION,
                     "compulsory_gbs": compulsory_gbs,
                     "compulsory_frac": (compulsory_gbs / HBM_PEAK_GBS) if compulsory_gbs else None,
                     "measured_copy_gbs": copy_gbs,
                     "timing": ("HIP events bracketing each solve's tier-launch graph replay on the launch "
                                "stream; avg launch = span / launches (includes in-graph gaps)"
                                if world == 1 else
                                "HIP events around rank 0's whole sharded solve (includes halo waits)")},
        "exchanged_bytes_per_step_rank0": st["exchanged_bytes"],
        "sharding": None if (world == 1 and args.virtual_ranks == 1) else {
            "halo_batch_tiers": args.dist_batch, "halo_batch_autotune_ms": autotune, "halo_slots": args.dist_slots,
            "halo_symmetric_fill": bool(args.dist_symmetry),
            "block_owner": ("split heaps in halves", "tier-balanced")[args.dist_owner],
            "host_enqueue_ms_per_step_rank0": enqueue_ms / max(1, args.steps),
            "per_rank_gpu_ms_and_enqueue_ms_per_step": per_rank},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_heaps)
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


if __name__ == "__main__":
    main()
