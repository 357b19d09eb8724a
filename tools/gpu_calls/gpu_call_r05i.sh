#!/bin/bash
# Round 5: split box engine op times dumped for offline schedule replays (B = 1, 2).
set -o pipefail
mkdir -p gpurun_out/r05i
for b in 1 2; do
    timeout -k 10 400 python -X faulthandler -u tools/box_split_time.py --ranks 2 4 8 --reps 3 --batch $b \
        --dump gpurun_out/r05i >> gpurun_out/r05i/split_time.txt 2>&1 || exit 1
done
