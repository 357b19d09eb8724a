#!/bin/bash
# Round 6: Othello 8x8 on the device (128-bit keys), and the sparse engines after the key-type
# templating (single-GPU parity, sharded loopback, IPC processes).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
P="python3 -u -m pytest -v --timeout 300 --timeout-method thread"
steps=(
  "600:r06d_othello8:$P tests/test_gpu_othello8.py"
  "400:r06d_sharded_sparse:$P tests/test_gpu_sharded.py -k sparse"
  "500:r06d_multiproc:$P tests/test_gpu_multiproc.py -k 'othello8 or sparse_ipc'"
  "900:r06d_parity:$P tests/test_gpu_parity.py"
)
tools/gpu_steps.sh "${steps[@]}"
