#!/bin/bash
mkdir -p gpurun_out/r04p
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 200 python tools/solve_timed.py toot 6 4 4 > gpurun_out/r04p/toot64.log 2>&1 || exit 1
timeout -k 10 200 python tools/solve_timed.py othello 4 4 4 > gpurun_out/r04p/oth.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -m gpu -x -v --timeout 240 --timeout-method thread -k "toot or othello or sparse or ttt" > gpurun_out/r04p/pytest_sparse.log 2>&1
