#!/bin/bash
mkdir -p gpurun_out/r04t
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for i in 1 2; do
GM_LIB_PATH=_exp/libgm_plainld.so timeout -k 10 180 python tools/box_shard_time.py --ranks 2 4 8 --reps 10 > gpurun_out/r04t/plain_$i.log 2>&1 || exit 1
timeout -k 10 180 python tools/box_shard_time.py --ranks 2 4 8 --reps 10 > gpurun_out/r04t/sc1_$i.log 2>&1 || exit 1
done
