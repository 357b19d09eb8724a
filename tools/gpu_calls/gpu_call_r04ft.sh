#!/bin/bash
# dataflow box launch: per-group trace at G = 8 and G = 1 (tools/flow_trace.py), and the
# poll sleep (GM_BOX_FLOW_SLEEP) against the per-rank G = 8 time
mkdir -p gpurun_out/r04ft
export PYTHONUNBUFFERED=1
GM_LIB_PATH=_exp/libgm_ftr.so GM_BOX_FLOW_TRACE_OUT=gpurun_out/r04ft/g8.bin timeout -k 10 120 python tools/box_shard_time.py --ranks 8 --reps 3 > gpurun_out/r04ft/trace_g8.log 2>&1 || exit 1
GM_BOX_FLOW=1 GM_LIB_PATH=_exp/libgm_ftr.so GM_BOX_FLOW_TRACE_OUT=gpurun_out/r04ft/g1.bin timeout -k 10 120 python tools/box_shard_time.py --ranks 1 --reps 3 > gpurun_out/r04ft/trace_g1.log 2>&1 || exit 1
for rep in 1; do
  for v in sl2 sl0 sl1 sl6; do
    GM_LIB_PATH=_exp/libgm_$v.so timeout -k 10 120 python tools/box_shard_time.py --ranks 8 --reps 10 > gpurun_out/r04ft/${v}_$rep.log 2>&1 || exit 1
  done
done
