#!/bin/bash
# round 5, first GPU call: the split box engine's GPU tests, smoke, per-rank timing
set -o pipefail
mkdir -p gpurun_out/r05a
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread -k "box" > gpurun_out/r05a/pytest_box.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05a/smoke.log 2>&1 &&
timeout -k 10 600 python -u tools/box_split_time.py --ranks 2 4 8 --reps 3 > gpurun_out/r05a/split_time.txt 2>&1
