#!/bin/bash
# Round 5: gm_query per engine, the bench at N = 1 and with 8 virtual ranks (split engine).
set -o pipefail
mkdir -p gpurun_out/r05e
timeout -k 10 300 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_abi.py tests/test_gpu_sharded.py -m gpu -k "query or region or custom" \
    > gpurun_out/r05e/pytest_abi.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r05e/bench.txt 2> gpurun_out/r05e/bench.err || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --virtual-ranks 8 --no-cpu-baseline --no-toot \
    > gpurun_out/r05e/bench_v8.txt 2> gpurun_out/r05e/bench_v8.err || exit 1
