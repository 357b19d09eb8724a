#!/bin/bash
# Round 5: split heaps -- the default (3 | 3,7 | 2,3,7) against A heaps only (2,3 | 1,2,3).
set -o pipefail
mkdir -p gpurun_out/r05q/def gpurun_out/r05q/a
timeout -k 10 400 python -X faulthandler -u tools/box_split_time.py --ranks 4 8 --reps 3 --batch 1 \
    --dump gpurun_out/r05q/def > gpurun_out/r05q/def.txt 2>&1 || exit 1
GM_BOX_SPLIT_HEAPS=2,3 timeout -k 10 300 python -X faulthandler -u tools/box_split_time.py --ranks 4 --reps 3 --batch 1 \
    --dump gpurun_out/r05q/a > gpurun_out/r05q/a4.txt 2>&1 || exit 1
GM_BOX_SPLIT_HEAPS=1,2,3 timeout -k 10 300 python -X faulthandler -u tools/box_split_time.py --ranks 8 --reps 3 --batch 1 \
    --dump gpurun_out/r05q/a > gpurun_out/r05q/a8.txt 2>&1 || exit 1
