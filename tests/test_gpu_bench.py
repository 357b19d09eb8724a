"""The bench.py contract on the GPU: one JSON line with the driver's fields, the roofline
and parity objects, at N = 1 and with 4 virtual ranks (the split box engine)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
          "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")


def _bench(*args):
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "3", "--warmup", "1", "--no-toot",
                        "--no-cpu-baseline", *args], capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_line_one_gpu():
    d = _bench()
    assert all(k in d for k in FIELDS)
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["value"] > 0 and d["parity"]["ok"]
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and 0 < rf["frac"] < 1 and rf["peak"] == 8000.0
    assert rf["launches_per_solve"] == 41 and rf["kernel"].startswith("box_tier_kernel<false>")


def test_bench_line_virtual_ranks_split():
    """4 virtual ranks: the split box engine -- every box on one rank (work_vs_one_gpu = 1),
    the ranks' tier launches, halo bytes per rank, parity of the whole table."""
    d = _bench("--virtual-ranks", "4")
    sh = d["sharding"]
    assert d["parity"]["ok"] and sh["boxes_per_rank"] == [262144] * 4 and sh["work_vs_one_gpu"] == 1.0
    assert sum(sh["halo_bytes_received_per_step_by_rank"]) > 0
    rf = d["roofline"]
    assert rf["launches_per_solve"] > 4 * 30 and rf["kernel"].startswith("box_tier_kernel<true>")
    assert rf["traffic"] is None   # the committed PMC summary is the one-GPU solve's


def test_bench_rehearsal_two_processes_one_gpu():
    """bench.py at N = 2 as the driver launches it (torch.distributed.run, one process per
    rank), both ranks on this one GPU (--rehearse-one-gpu: gloo for the bench's collectives,
    the IPC transport for the halos): the IPC probe passes (no fallback), every rank's owned
    digest equals the oracle's, the side configs shard over the sparse IPC transport, and the
    line says it is a rehearsal."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29531", os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--rehearse-one-gpu", "--dist-batch", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, cwd=REPO)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["parity"]["ok"] and d["halo_transport_fallback"] is None
    assert d["rehearsal"] and d["sharding"]["work_vs_one_gpu"] == 1.0
    assert d["parity"]["per_rank_vs_oracle"]["wrong_ranks"] == []
    # the side configs' hash-sharded solves at N = 2, over the sparse IPC transport (RCCL refuses
    # two ranks on one GPU): summed digests, counts and root records equal the oracle's
    oc = d["other_configs"]
    for name in ("othello_4x4", "toot_6x4"):
        assert oc[name]["ok"] and oc[name]["ranks"] == 2 and "IPC" in oc[name]["transport"], oc[name]
    assert oc["toot_6x4"]["symmetry_off"]["digest_matches_oracle"]


def test_bench_rehearsal_failed_probe_exits_cleanly():
    """a rehearsal whose IPC probe fails (forced by the GM_BENCH_PROBE_FAIL
    hook) has nothing to fall back to, so bench.py ends at once with status 4 and one JSON
    error line -- no autotune or timed solves on the broken transport, no traceback cascade."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29533", os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--rehearse-one-gpu", "--dist-batch", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, cwd=REPO,
                       env=dict(os.environ, GM_BENCH_PROBE_FAIL="1"))
    assert r.returncode != 0
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["value"] is None and "probe failed" in d["error"]
    assert 'bench.py", line' not in r.stderr, r.stderr[-3000:]   # no traceback through bench.py (torchrun
    # itself reports the failed child with its own traceback)
