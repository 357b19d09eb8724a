"""Drive the reference's live engine (``src/new_process.py``) on one fake-MPI rank.

Build-container only (called by ``make_golden.py --live``).  The engine's job loop
(``Process.run``, ``src/new_process.py:37-60``) runs unmodified; ``comm``,
``isend``, ``recv`` and ``abort`` are replaced by an in-process mailbox, and the
``abort`` the root calls after printing its line (``:53``) ends the run.  The
engine's ``resolved``/``remote`` shelve tables are then compared with the
canonical table: values must agree everywhere; remoteness is expected to differ
by -1 on some positions (``gs_tup`` captured before the primitive
remoteness is set, ``src/new_process.py:108`` vs ``:122-123``).
"""
import importlib
import io
import os
import sys
import tempfile
import time
import contextlib

REF = "/root/reference"


class _Done(Exception):
    pass


class _Req:
    def test(self):
        return True, None


class _Comm:
    def __init__(self):
        self.box = []

    def isend(self, job, dest=0):
        self.box.append(job)
        return _Req()

    def recv(self):
        return self.box.pop(0)

    def Iprobe(self):
        return bool(self.box)

    def Abort(self):
        raise _Done()


def _fresh_engine(ref_utils, module):
    ref_utils.game_module = module
    for name in ("src.game_state", "src.new_job", "src.new_process", "src.cache_dict"):
        sys.modules.pop(name, None)
    gs = importlib.import_module("src.game_state")
    job = importlib.import_module("src.new_job")
    proc = importlib.import_module("src.new_process")
    return gs, job, proc


def run_live(ref_utils, module, root=None):
    if root is not None:
        module.initial_position = lambda r=root: r
    gs, job_mod, proc_mod = _fresh_engine(ref_utils, module)
    comm = _Comm()
    with tempfile.TemporaryDirectory() as sd:
        cwd = os.getcwd()
        os.chdir(sd)
        try:
            p = proc_mod.Process(0, 1, comm, comm.isend, comm.recv, comm.Abort, stats_dir=sd)
            init = gs.GameState(gs.GameState.INITIAL_POS)
            p.work.put(job_mod.Job(job_mod.Job.LOOK_UP, 0, job_mod.Job.INITIAL_JOB_ID,
                                   init.to_tuple()))
            out = io.StringIO()
            t0 = time.time()
            with contextlib.redirect_stdout(out):
                try:
                    p.run()
                except _Done:
                    pass
            secs = time.time() - t0
            resolved = {k: p.resolved._file_dict[k] for k in p.resolved._file_dict.keys()}
            remote = {k: p.remote._file_dict[k] for k in p.remote._file_dict.keys()}
        finally:
            os.chdir(cwd)
            proc_mod.Process.IS_FINISHED = False
    return out.getvalue().strip(), resolved, remote, secs


def compare(canon_table, canon_positions, resolved, remote):
    by_str = {str(canon_positions[k]): v for k, v in canon_table.items()}
    val_bad = rem_bad = 0
    deltas = {}
    for s, v in resolved.items():
        cv, cr = by_str[s]
        if v != cv:
            val_bad += 1
        d = remote[s] - cr
        if d:
            rem_bad += 1
            deltas[d] = deltas.get(d, 0) + 1
    return {"positions_live": len(resolved), "positions_canonical": len(canon_table),
            "value_mismatches": val_bad, "remoteness_mismatches": rem_bad,
            "remoteness_deltas": {str(k): v for k, v in sorted(deltas.items())}}


def run_all(load, canonical, ref_utils):
    out = {}
    f2o = load("game_module", os.path.join(REF, "test_games/four_to_one.py"))
    for root in ("4", "6", "1", "0"):
        f2o = load("game_module", os.path.join(REF, "test_games/four_to_one.py"))
        line, res, rem, secs = run_live(ref_utils, f2o, root)
        f2o = load("game_module", os.path.join(REF, "test_games/four_to_one.py"))
        t, pos = canonical.solve(f2o, root)
        entry = compare(t, pos, res, rem)
        entry.update(root_line_live=line, seconds=round(secs, 2))
        out["four_to_one/%s" % root] = entry
    mttt = load("game_module", os.path.join(REF, "test_games/mttt.py"))
    line, res, rem, secs = run_live(ref_utils, mttt)
    t, pos = canonical.solve(mttt)
    entry = compare(t, pos, res, rem)
    entry.update(root_line_live=line, seconds=round(secs, 2))
    out["mttt"] = entry
    oth = load("game_module", os.path.join(REF, "test_games/othello_bit_new.py"))
    oth.length, oth.height, oth.area = 4, 4, 16
    line, res, rem, secs = run_live(ref_utils, oth)
    t, pos = canonical.solve(oth)
    entry = compare(t, pos, res, rem)
    entry.update(root_line_live=line, seconds=round(secs, 2))
    out["othello_4x4"] = entry
    return out
