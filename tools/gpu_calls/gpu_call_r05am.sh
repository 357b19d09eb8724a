#!/bin/bash
# Round 5: solo spans and DAG model of the IPC-emulated split (GM_BOX_SIGNAL_KERNELS=1) after the
# hand-off experiment was reverted, twice.
set -o pipefail
mkdir -p gpurun_out/r05am
for k in 1 2; do
  GM_BOX_SIGNAL_KERNELS=1 timeout -k 10 300 python -X faulthandler -u tools/box_split_time.py --ranks 2 4 8 --reps 3 --batch 1 \
      > gpurun_out/r05am/split_time_sigk$k.txt 2>&1 || exit 1
done
