#!/bin/bash
mkdir -p gpurun_out/r04o
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 180 python tools/box_shard_time.py --ranks 2 4 8 --reps 10 > gpurun_out/r04o/flow_drainflags.log 2>&1 || exit 1
GM_BOX_FLOW=1 timeout -k 10 120 python tools/box_shard_time.py --ranks 1 --reps 10 > gpurun_out/r04o/flow1_drainflags.log 2>&1 || exit 1
