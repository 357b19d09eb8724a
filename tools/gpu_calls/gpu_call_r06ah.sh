#!/bin/bash
# Round 6: the sparse IPC transport pulls with a copy kernel reading the peer's mapping (not
# hipMemcpyAsync): the multi-process sparse tests, then Toot 6x4 over 2 processes (symmetric).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06ah
steps=(
  "500:r06ah/multiproc:python3 -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_multiproc.py -k 'sparse or othello8 or toot'"
  "200:r06ah/toot64_ipc2:GM_TRACE=0 python3 -u tools/ipc_toot_probe.py 6 4 2 3 0"
)
tools/gpu_steps.sh "${steps[@]}"
