#!/bin/bash
# Round 6: the IPC stall -- Toot 6x4 over 2 processes, ONE solve without the symmetry reduction in
# fresh processes (r06ae stalled in that solve after two with the reduction).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06ak
timeout -k 10 170 python3 -u tools/ipc_toot_probe.py 6 4 2 0 1 > gpurun_out/r06ak/toot64_symoff_alone.log 2>&1; echo "rc=$?"
grep -v "hipMalloc\|pulls" gpurun_out/r06ak/toot64_symoff_alone.log | tail -8
