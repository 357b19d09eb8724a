#!/bin/bash
# sparse engine on Toot 6x4: sort bits scan (sorted lists, plain kernels)
mkdir -p gpurun_out/r04f
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
GM_SPARSE_BATCH=0 timeout -k 10 200 python tools/solve_timed.py toot 6 4 4 > gpurun_out/r04f/toot64_nosort.log 2>&1 || exit 1
for b in 8 16 24 32 48; do
  GM_SPARSE_SORT_BITS=$b timeout -k 10 200 python tools/solve_timed.py toot 6 4 4 > gpurun_out/r04f/toot64_bits$b.log 2>&1 || exit 1
done
GM_SPARSE_SORT_BITS=16 timeout -k 10 200 python tools/solve_timed.py othello 4 4 4 > gpurun_out/r04f/oth.log 2>&1 || exit 1
GM_SPARSE_SORT_BITS=16 timeout -k 10 200 python tools/solve_timed.py toot 5 4 4 > gpurun_out/r04f/toot54.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r04f/pytest_gpu.log 2>&1
