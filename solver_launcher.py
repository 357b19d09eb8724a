#!/usr/bin/env python3
"""Drop-in for the reference's ``solver_launcher.py`` (GamesmanMPI), solving on MI355X.

    python solver_launcher.py GAME_FILE [--debug] [-sd DIR] [--custom FILE --init_pos NAME] [--cp]
    python -m torch.distributed.run --nproc-per-node N solver_launcher.py GAME_FILE ...

Same arguments and the same single stdout line as the reference
(``"<WIN|LOSS|TIE> in <R> moves"``, printed by the root rank,
reference src/new_process.py:47-52).  The reference's flags are at
solver_launcher.py:9-41; the plugin is loaded by path and published as
``src.utils.game_module`` (:56-57) and checked with ``validate`` (:70-81).

Differences, on purpose:
* ``--custom/--init_pos`` takes effect (the reference freezes the root at import,
  src/game_state.py:15, so it silently ignores them -- SURVEY §0.3);
* the solve runs in libgmsolve.so on the GPU; ranks come from
  torch.distributed.run's environment instead of mpiexec.  With one GPU per rank
  the ranks shard the solve (RCCL); with more ranks than GPUs -- the reference's
  own tests run ``mpiexec --oversubscribe -n 2`` on one host
  (game_tests/four_to_one_test.py:20) -- rank 0 solves for all of them, running
  the same sharded algorithm over ``world`` loopback ranks on its GPU, and the
  other ranks wait at a barrier and exit 0.  Either way the root line is printed
  once.  Values and remoteness are the canonical ones;
* ``-sd DIR`` writes the solved table in the reference's layout -- shelve
  databases ``DIR/stats/<rank>/resolved`` and ``remote`` keyed by ``str(pos)``,
  each position on rank ``md5(str(pos)) % world`` (src/cache_dict.py:19-42,
  gamesmanmpi_amd/persist.py) -- and as ``DIR/stats/<rank>/table.npz`` (sorted
  u64 keys + u16 records); ``--sd-format`` picks one (shelves are written for
  tables of up to 2 million positions unless asked for explicitly);
* extras: ``--dims LxH`` patches board plugins' ``length``/``height``, ``--heaps``
  patches the subtraction plugin, ``--engine``, ``--device``, ``--stats``.
"""
import argparse
import cProfile
import importlib.util
import json
import logging
import os
import sys

REPO = os.path.dirname(os.path.abspath(__file__))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

import src.utils  # noqa: E402


SHELVE_AUTO_LIMIT = 2_000_000


def build_parser():
    p = argparse.ArgumentParser()
    p.add_argument("game_file", help="Game to solve for.")
    p.add_argument("--debug", help="Enables or disables logging.", action="store_true")
    p.add_argument("-sd", "--statsdir", help="Location to store statistics about game.", action="store")
    p.add_argument("--custom", help="Specifies custom file to modify provided game file.")
    p.add_argument("--init_pos", help="Initial position to start at for the game. "
                   "If none is specified, the default is used.")
    p.add_argument("--cp", action="store_true")
    p.add_argument("--dims", help="board plugins: LxH (sets the module's length/height)")
    p.add_argument("--heaps", type=int, help="subtraction plugin: number of heaps")
    p.add_argument("--engine", choices=("auto", "dense", "sparse"), default="auto")
    p.add_argument("--device", type=int, default=None)
    p.add_argument("--stats", action="store_true", help="print solve statistics (JSON) to stderr")
    p.add_argument("--sd-format", choices=("auto", "npz", "reference", "both"), default="auto",
                   help="-sd output: npz table, the reference's shelve layout, or both (auto: both up to "
                        "%d positions, else npz)" % SHELVE_AUTO_LIMIT)
    return p


def load_module(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    if spec is None:
        raise FileNotFoundError(path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def validate(mod):
    """The four plugin functions must exist (reference solver_launcher.py:70-81)."""
    for attr in ("initial_position", "do_move", "gen_moves", "primitive"):
        if not hasattr(mod, attr):
            print("Could not find method", attr)
            raise AttributeError(attr)


def custom_root(game, custom_path, name):
    """Initial position from ``--custom FILE --init_pos NAME`` (reference :83-111)."""
    try:
        custom = load_module("custom", custom_path)
    except (FileNotFoundError, OSError):
        print("Custom file was not found. Using default initial position instead.")
        return None
    except AttributeError:
        print("Custom file with new initial position not specified. "
              "Using default initial position instead.")
        return None
    fn = getattr(custom, name, None)
    if fn is None:
        print("Initial position was not found in custom file. Using default initial position instead.")
        return None
    game.initial_position = fn
    return fn()


def prepare_game(args):
    game = load_module("game_module", args.game_file)
    src.utils.game_module = game
    if args.dims:
        L, H = (int(v) for v in args.dims.lower().split("x"))
        game.length, game.height = L, H
        if hasattr(game, "area"):
            game.area = L * H
    if args.heaps is not None:
        game.HEAPS = args.heaps
    validate(game)
    root = None
    if args.init_pos:
        root = custom_root(game, args.custom, args.init_pos)
    if root is None:
        root = game.initial_position()
    return game, root


def dist_env():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


MAX_VIRTUAL_RANKS = 64   # GM_OPT_VIRTUAL_RANKS range (include/gmsolve.h)


def rank_plan(world, local_world, n_devices):
    """How `world` launcher ranks share the solve (the reference's mpiexec -n N).

    "solo"     one rank: it solves;
    "sharded"  one GPU per rank on one node: every rank joins the RCCL solve;
    "single"   more ranks than GPUs (mpiexec --oversubscribe): rank 0 solves for all,
               the others wait at a barrier and exit 0."""
    if world <= 1:
        return "solo"
    if local_world == world and world <= n_devices:
        return "sharded"
    return "single"


def run(args, out=sys.stdout):
    rank, world, local = dist_env()
    if args.debug:
        os.makedirs("logs", exist_ok=True)
        logging.basicConfig(filename="logs/proc%d" % rank, level=logging.DEBUG)
    game, root = prepare_game(args)

    from gamesmanmpi_amd import Solver, _lib
    plan = "solo"
    if world > 1:
        from gamesmanmpi_amd import dist
        dist.init_group()
        plan = dist.broadcast(rank_plan(world, int(os.environ.get("LOCAL_WORLD_SIZE", world)),
                                        _lib.lib().gm_device_count()) if rank == 0 else None)
        logging.debug("rank %d of %d: %s", rank, world, plan)
        if plan == "single" and rank != 0:
            # rank 0 solves for every rank and prints the root line; wait for it by polling
            # the group's store (a barrier would time out under a solve longer than the
            # group timeout)
            return dist.wait_for_root()
    if plan == "single":
        try:
            return _solve_and_report(args, game, root, rank, world, local, plan, out)
        except BaseException:
            dist.release_waiters(world, ok=False)
            raise
    return _solve_and_report(args, game, root, rank, world, local, plan, out)


def _solve_and_report(args, game, root, rank, world, local, plan, out):
    from gamesmanmpi_amd import Solver, _lib
    if world > 1:
        from gamesmanmpi_amd import dist
    engine = {"auto": None, "dense": _lib.ENGINE_DENSE, "sparse": _lib.ENGINE_SPARSE}[args.engine]
    device = args.device if args.device is not None else (local if plan == "sharded" else -1)
    solver = Solver(game, root, device=device, engine=engine)
    if plan == "sharded":
        dist.join(solver.ctx, rank, world)
    elif plan == "single" and solver.codec.game_id != _lib.GAME_GRAPH and world <= MAX_VIRTUAL_RANKS:
        # the sharded algorithm over `world` loopback ranks on this one GPU
        solver.ctx.set_option(_lib.OPT_VIRTUAL_RANKS, world)
    logging.debug("solving %s from %r on device %s", args.game_file, root, device)
    if args.cp:
        prof = cProfile.Profile()
        prof.runcall(solver.solve)
        prof.dump_stats("time")
    else:
        solver.solve()
    if rank == 0:
        out.write(solver.root_line() + "\n")
        out.flush()
    if args.stats:
        st = solver.ctx.stats()
        st["rank"] = rank
        print(json.dumps(st), file=sys.stderr)
    if args.statsdir:
        write_statsdir(args, solver, rank, world, gather=plan == "sharded")
    solver.close()
    if plan == "single":
        dist.release_waiters(world)
    return 0


def write_statsdir(args, solver, rank, world, gather=True):
    """-sd DIR: this rank's npz table and/or the reference's shelve layout (rank 0
    writes every rank's shelves, gathering the sharded ranks' tables first; with
    gather False rank 0 holds the whole table)."""
    from gamesmanmpi_amd.persist import write_reference_tables
    from gamesmanmpi_amd.solver import dump_table
    keys, recs = solver.table()
    fmt = args.sd_format
    if fmt == "auto":
        total = solver.n_positions or len(keys)
        fmt = "both" if total <= SHELVE_AUTO_LIMIT else "npz"
        if fmt == "npz" and rank == 0:
            print("-sd: %d positions; writing table.npz only (--sd-format reference forces the shelves)" % total,
                  file=sys.stderr)
    if fmt in ("npz", "both"):
        dump_table(os.path.join(args.statsdir, "stats", str(rank), "table.npz"), keys, recs,
                   {"game": args.game_file, "codec": solver.codec.name, "params": solver.codec.params})
    if fmt in ("reference", "both"):
        if world > 1 and gather:
            import numpy as np
            import torch.distributed as tdist
            parts = [None] * world
            tdist.all_gather_object(parts, (keys, recs))
            keys = np.concatenate([p[0] for p in parts])
            recs = np.concatenate([p[1] for p in parts])
        if rank == 0:
            write_reference_tables(args.statsdir, solver.codec, keys, recs, world)


def main(argv=None):
    args = build_parser().parse_args(argv)
    return run(args)


if __name__ == "__main__":
    sys.exit(main())
