#!/bin/bash
# round 5: per-rank split-box timing (held eager solo), batch sizes 1/2/4, comparisons for reference
set -o pipefail
mkdir -p gpurun_out/r05b
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 200 --timeout-method thread -k "solo_timing" > gpurun_out/r05b/pytest_solo.log 2>&1 &&
for b in 1 2 4; do timeout -k 10 400 python -X faulthandler -u tools/box_split_time.py --ranks 2 4 8 --reps 3 --batch $b >> gpurun_out/r05b/split_time.txt 2>&1 || exit 1; done &&
timeout -k 10 400 python -X faulthandler -u tools/box_split_time.py --ranks 2 4 8 --reps 3 --batch 1 --split 1 >> gpurun_out/r05b/split_time.txt 2>&1
