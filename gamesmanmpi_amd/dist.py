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
import os
import sys

from . import _lib


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


def init_group(backend="gloo"):
    """The launcher's process group (host side only: gloo touches no GPU); the
    rendezvous comes from torch.distributed.run's MASTER_ADDR / MASTER_PORT."""
    import torch.distributed as tdist
    if not tdist.is_initialized():
        with quiet_stdout():
            tdist.init_process_group(backend)
    return tdist


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
