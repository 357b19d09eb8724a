#!/bin/bash
mkdir -p gpurun_out/r04w
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 200 python tools/solve_timed.py toot 6 4 4 > gpurun_out/r04w/toot64.log 2>&1 || exit 1
timeout -k 10 200 python tools/solve_timed.py othello 4 4 4 > gpurun_out/r04w/oth.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04w/kt -o run -- python3 tools/solve_timed.py toot 6 4 3 > gpurun_out/r04w/kt.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_graph.py -m gpu -x -v --timeout 240 --timeout-method thread -k "toot or othello or sparse or ttt or four or graph" > gpurun_out/r04w/pytest_sparse.log 2>&1
