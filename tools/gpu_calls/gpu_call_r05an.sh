#!/bin/bash
# Round 5: the bench GPU tests, including the two-process rehearsal on one GPU.
set -o pipefail
mkdir -p gpurun_out/r05an
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bench.py \
    > gpurun_out/r05an/pytest_bench.txt 2>&1 || exit 1
