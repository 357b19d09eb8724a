"""Multi-GPU bootstrap: one process per GPU, ranks from torch.distributed.run.

Replaces the reference's ``mpi4py.MPI.COMM_WORLD`` set-up
(solver_launcher.py:47-52): rank 0 creates an RCCL unique id through the C ABI
(``gm_comm_unique_id``), every rank receives it over a torch.distributed group
(gloo by default: the bootstrap touches no GPU), and each context joins the RCCL
communicator with ``gm_set_comm``.  All data-path exchange then happens inside
libgmsolve.so (RCCL over xGMI).
"""
import contextlib
import ctypes
import datetime
import os
import sys
import time

from . import _lib

# Timeout of the launcher's gloo group (seconds; GM_DIST_TIMEOUT_S).  torch's default of
# 30 minutes is shorter than a long solve plus -sd writes, and a collective that times
# out ends the rank; torchrun ends every rank when one fails, so a long default costs
# nothing when a rank dies.
DEFAULT_TIMEOUT_S = 7 * 24 * 3600.0
DONE_KEY, ACK_KEY = "gm_launcher_root_done", "gm_launcher_ack"


def group_timeout_s():
    return float(os.environ.get("GM_DIST_TIMEOUT_S", DEFAULT_TIMEOUT_S))


@contextlib.contextmanager
def quiet_stdout():
    """Send file descriptor 1 to stderr while the gloo group connects: gloo prints
    "[Gloo] Rank r is connected to ..." on stdout, and the launcher's stdout must be
    exactly the reference's root line (game_tests/four_to_one_test.py:23)."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def unique_id():
    buf = ctypes.create_string_buffer(128)
    _lib.check(_lib.lib().gm_comm_unique_id(buf, 128))
    return buf.raw


def init_group(backend="gloo", timeout_s=None):
    """The launcher's process group (host side only: gloo touches no GPU); the
    rendezvous comes from torch.distributed.run's MASTER_ADDR / MASTER_PORT, the
    timeout from GM_DIST_TIMEOUT_S (default a week) instead of torch's 30 minutes."""
    import torch.distributed as tdist
    if not tdist.is_initialized():
        with quiet_stdout():
            tdist.init_process_group(backend, timeout=datetime.timedelta(
                seconds=timeout_s if timeout_s is not None else group_timeout_s()))
    return tdist


def _store():
    from torch.distributed import distributed_c10d as c10d
    return c10d._get_default_store()


def wait_for_root(poll_s=0.2, timeout_s=None):
    """A rank with nothing to solve (more ranks than GPUs: rank 0 solves for all) waits for
    rank 0's result by polling the group's key-value store, not in a collective, so a solve
    that outlasts the group timeout does not end the waiting ranks (GM_DIST_WAIT_S sets a
    deadline; none by default).  Returns 0, or 1 if rank 0 reports a failure."""
    store = _store()
    if timeout_s is None and os.environ.get("GM_DIST_WAIT_S"):
        timeout_s = float(os.environ["GM_DIST_WAIT_S"])
    t0 = time.monotonic()
    while not store.check([DONE_KEY]):   # no deadline by default: rank 0 posts failures too
        if timeout_s is not None and time.monotonic() - t0 > timeout_s:
            raise TimeoutError("rank 0 did not finish the solve within %.0f s" % timeout_s)
        time.sleep(poll_s)
    ok = store.get(DONE_KEY) == b"ok"
    store.add(ACK_KEY, 1)
    return 0 if ok else 1


def release_waiters(world, ok=True, timeout_s=60.0):
    """Rank 0: post the solve's outcome for wait_for_root and wait (briefly) until every
    waiting rank has read it, so the store outlives their last poll."""
    store = _store()
    store.set(DONE_KEY, "ok" if ok else "error")
    deadline = time.monotonic() + timeout_s
    while store.add(ACK_KEY, 0) < world - 1 and time.monotonic() < deadline:
        time.sleep(0.05)


def broadcast(obj, src=0):
    """`obj` of rank `src` on every rank (reference: comm.bcast)."""
    box = [obj]
    g = init_group()
    with quiet_stdout():
        g.broadcast_object_list(box, src=src)
    return box[0]


def barrier():
    """All ranks (reference solver_launcher.py:60,114,166 comm.Barrier)."""
    g = init_group()
    with quiet_stdout():
        g.barrier()


def share_unique_id(rank, backend="gloo"):
    init_group(backend)
    return broadcast(unique_id() if rank == 0 else None)


def join(ctx, rank, world, backend="gloo"):
    """Make ``ctx`` (a solver.Context) one rank of a ``world``-GPU solve."""
    uid = share_unique_id(rank, backend) if world > 1 else None
    ctx.set_comm(rank, world, uid)
    return uid
