#!/bin/bash
mkdir -p gpurun_out/r04m
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
GM_BOX_FLOW=1 timeout -k 10 180 python tools/box_shard_time.py --ranks 1 2 4 8 --reps 10 > gpurun_out/r04m/flow3.log 2>&1 || exit 1
GM_BOX_FLOW=1 GM_BOX_FLOW_ORDER=0 timeout -k 10 180 python tools/box_shard_time.py --ranks 1 2 4 8 --reps 10 > gpurun_out/r04m/flow3_hilbert.log 2>&1 || exit 1
