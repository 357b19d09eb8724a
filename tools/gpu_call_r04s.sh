#!/bin/bash
mkdir -p gpurun_out/r04s
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for i in 1 2; do
GM_BOX_FLOW_DYN=1 timeout -k 10 180 python tools/box_shard_time.py --ranks 2 4 8 --reps 10 > gpurun_out/r04s/dyn_$i.log 2>&1 || exit 1
GM_BOX_FLOW_DYN=0 timeout -k 10 180 python tools/box_shard_time.py --ranks 2 4 8 --reps 10 > gpurun_out/r04s/static_$i.log 2>&1 || exit 1
done
