"""Run one function per rank in spawned processes, and never leave one behind.

Used by the multi-process RCCL tests (tests/test_gpu_multiproc.py) and tested on
the CPU with gloo ranks (tests/test_dist_plan.py).  Every rank reports its phases
("start", "comm", "solve", ...) to the parent.  On a deadline, a rank error or a
rank that dies, the parent terminates every rank (SIGTERM), kills what is left
after a grace period (SIGKILL), and raises RankFailure naming each rank's last
phase -- so a hung exchange ends the test instead of holding GPUs.
"""
import multiprocessing as mp
import queue
import time


class RankFailure(AssertionError):
    pass


def _entry(target, rank, world, args, q):
    def phase(name):
        q.put(("phase", rank, name))
    phase("start")
    try:
        res = target(rank, world, phase, *args)
        q.put(("done", rank, res))
    except BaseException as e:  # reported to the parent, which stops every rank
        q.put(("error", rank, "%s: %s" % (type(e).__name__, e)))


def run_ranks(target, world, args=(), timeout=240.0, grace=10.0):
    """target(rank, world, phase, *args) -> picklable result, in `world` processes.
    Returns the results by rank, or raises RankFailure after stopping every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_entry, args=(target, r, world, args, q), daemon=True) for r in range(world)]
    for p in procs:
        p.start()
    last = {r: "spawned" for r in range(world)}
    results, errors = {}, {}
    deadline = time.monotonic() + timeout
    why = None
    try:
        while len(results) < world:
            left = deadline - time.monotonic()
            if left <= 0:
                why = "timeout after %.0f s" % timeout
                break
            try:
                kind, rank, val = q.get(timeout=min(1.0, left))
            except queue.Empty:
                dead = [r for r, p in enumerate(procs) if p.exitcode is not None and r not in results]
                if dead:
                    # a rank may have exited just after queueing its result: drain once more
                    time.sleep(0.2)
                    try:
                        while True:
                            kind, rank, val = q.get_nowait()
                            if kind == "done":
                                results[rank] = val
                            elif kind == "error":
                                errors[rank] = val
                            else:
                                last[rank] = val
                    except queue.Empty:
                        pass
                    dead = [r for r in dead if r not in results]
                    if dead:
                        why = "rank(s) %s exited with %s" % (dead, [procs[r].exitcode for r in dead])
                        break
                continue
            if kind == "phase":
                last[rank] = val
            elif kind == "done":
                results[rank] = val
                last[rank] = "done"
            else:
                errors[rank] = val
                why = "rank %d failed: %s" % (rank, val)
                break
    finally:
        stop(procs, grace)
    if why is not None or errors:
        raise RankFailure("%s; last phase per rank: %s; errors: %s"
                          % (why, ", ".join("%d=%s" % (r, last[r]) for r in range(world)), errors))
    return [results[r] for r in range(world)]


def stop(procs, grace=10.0):
    """SIGTERM every live process, SIGKILL what is left after `grace` seconds, reap all."""
    for p in procs:
        if p.is_alive():
            p.terminate()
    t = time.monotonic() + grace
    for p in procs:
        p.join(timeout=max(0.0, t - time.monotonic()))
    for p in procs:
        if p.is_alive():
            p.kill()
            p.join(timeout=5)
