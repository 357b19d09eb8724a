#!/bin/bash
# Round 6: Toot 6x4 over 2 processes sharing one GPU on the sparse IPC transport, two solves with
# the symmetry reduction and one without, in the same contexts (the order bench.py's side config
# uses; r06ad stalled in the third), traced per tier.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06ae
timeout -k 10 150 python3 -u tools/ipc_toot_probe.py 6 4 2 2 1 > gpurun_out/r06ae/toot64.log 2>&1; echo "rc=$?"
grep -v "hipMalloc\|ipc rank" gpurun_out/r06ae/toot64.log | tail -12
