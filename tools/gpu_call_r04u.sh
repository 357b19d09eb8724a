#!/bin/bash
mkdir -p gpurun_out/r04u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
GM_BOX_FLOW=0 timeout -k 10 120 python tools/box_shard_time.py --ranks 1 --reps 10 > gpurun_out/r04u/tiers.log 2>&1
GM_BOX_FLOW=2 timeout -k 10 120 python tools/box_shard_time.py --ranks 1 --reps 10 > gpurun_out/r04u/nowait.log 2>&1
GM_BOX_FLOW=3 timeout -k 10 120 python tools/box_shard_time.py --ranks 1 --reps 10 > gpurun_out/r04u/nowait_nopub.log 2>&1
GM_LIB_PATH=_exp/libgm_plainld.so GM_BOX_FLOW=3 timeout -k 10 120 python tools/box_shard_time.py --ranks 1 --reps 10 > gpurun_out/r04u/nowait_nopub_plain.log 2>&1
GM_BOX_FLOW=1 timeout -k 10 120 python tools/box_shard_time.py --ranks 1 --reps 10 > gpurun_out/r04u/flow.log 2>&1
exit 0
