#!/bin/bash
# Round 6: the sparse IPC transport through one fixed window per rank: the multi-process tests,
# then Toot 6x4 over 2 processes -- two solves with the symmetry reduction, one without (the
# solve that stalled in r06ae / r06ak) -- and over 3 processes.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06am
steps=(
  "500:r06am/multiproc:python3 -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_multiproc.py"
  "250:r06am/toot64_ipc2:GM_TRACE=0 python3 -u tools/ipc_toot_probe.py 6 4 2 2 1"
  "250:r06am/toot64_ipc3:GM_TRACE=0 python3 -u tools/ipc_toot_probe.py 6 4 3 1 1"
)
tools/gpu_steps.sh "${steps[@]}"
