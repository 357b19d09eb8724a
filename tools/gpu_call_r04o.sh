#!/bin/bash
mkdir -p gpurun_out/r04o
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for i in 1 2; do
GM_BOX_FLOW_WINDOW=1 timeout -k 10 180 python tools/box_shard_time.py --ranks 2 4 8 --reps 10 > gpurun_out/r04o/win1_$i.log 2>&1 || exit 1
GM_BOX_FLOW_WINDOW=0 timeout -k 10 180 python tools/box_shard_time.py --ranks 2 4 8 --reps 10 > gpurun_out/r04o/win0_$i.log 2>&1 || exit 1
done
