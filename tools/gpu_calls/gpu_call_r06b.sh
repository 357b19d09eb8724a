#!/bin/bash
# Round 6: the sparse engine's IPC transport across processes (ranks sharing the GPU), the box
# engine's poisoned IPC tests and the early-read fault hook, the bench's probe / rehearsal.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
P="python3 -u -m pytest -v --timeout 240 --timeout-method thread"
steps=(
  "500:r06b_sparse_ipc:$P tests/test_gpu_multiproc.py -k sparse_ipc"
  "700:r06b_box_ipc:$P tests/test_gpu_multiproc.py -k box_ipc"
  "600:r06b_bench:$P tests/test_gpu_bench.py"
)
tools/gpu_steps.sh "${steps[@]}"
