#!/bin/bash
# debug: sparse batch path (sorted interior lists), no test may leave a fault behind
mkdir -p gpurun_out/r04d
export PYTHONUNBUFFERED=1
GM_SPARSE_BATCH=3 timeout -k 10 200 python tools/solve_timed.py toot 5 4 1 > gpurun_out/r04d/toot54_m3.log 2>&1 &&
GM_SPARSE_BATCH=3 timeout -k 10 200 python tools/solve_timed.py toot 6 4 1 > gpurun_out/r04d/toot64_m3.log 2>&1 &&
GM_TRACE=1 timeout -k 10 200 python tools/solve_timed.py toot 5 4 2 > gpurun_out/r04d/toot54_m1.log 2>&1 &&
GM_TRACE=1 timeout -k 10 200 python tools/solve_timed.py toot 6 4 2 > gpurun_out/r04d/toot64_m1.log 2>&1
