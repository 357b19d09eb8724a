#!/bin/bash
# Round 5: the split box engine across processes with the IPC transport (ranks sharing the GPU).
set -o pipefail
mkdir -p gpurun_out/r05k
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multiproc.py -k "ipc" \
    > gpurun_out/r05k/pytest_ipc.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_sharded.py -k "box" \
    > gpurun_out/r05k/pytest_box.txt 2>&1 || exit 1
