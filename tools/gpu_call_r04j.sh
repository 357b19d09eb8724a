#!/bin/bash
mkdir -p gpurun_out/r04j
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for i in 1 2 3; do
for v in "256 5000" "64 5000" "256 500" "64 500"; do set -- $v
GM_GRAPH_CHUNK=$1 GM_GRAPH_SWITCH_US=$2 timeout -k 10 100 python tools/graph_enum_time.py 16 16 > gpurun_out/r04j/g_c$1_s$2_$i.log 2>&1 || exit 1
done; done
