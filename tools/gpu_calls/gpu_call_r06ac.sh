#!/bin/bash
# Round 6: Toot 6x4 over 2 processes sharing one GPU on the sparse IPC transport, traced per tier
# (the rehearsal's side config did not finish within 240 s in r06ab).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06ac
timeout -k 10 300 python3 -u tools/ipc_toot_probe.py 5 4 2 2 > gpurun_out/r06ac/toot54.log 2>&1; echo "rc54=$?"
timeout -k 10 300 python3 -u tools/ipc_toot_probe.py 6 4 2 1 > gpurun_out/r06ac/toot64.log 2>&1; echo "rc64=$?"
tail -5 gpurun_out/r06ac/toot54.log; tail -30 gpurun_out/r06ac/toot64.log
