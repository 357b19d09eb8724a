#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05c
for b in 1 4; do timeout -k 10 400 python -X faulthandler -u tools/box_split_time.py --ranks 8 --reps 3 --batch $b >> gpurun_out/r05c/split_kinds.txt 2>&1 || exit 1; done
