#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
steps=()
for t in serp serp0 plain; do
  steps+=("60:$t:GM_WK_MIN=0 GM_LIB_PATH=_exp/libgm_$t.so python -u tools/quick_time.py 3,256,10,2 3,256,10,2")
  steps+=("90:f_$t:GM_WK_MIN=0 GM_LIB_PATH=_exp/libgm_$t.so timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/f_$t -o run -- python3 tools/quick_time.py 3,256,10,2")
done
steps+=("60:def:GM_WK_MIN=0 python -u tools/quick_time.py 3,256,10,2 3,256,10,2")
steps+=("90:f_def:GM_WK_MIN=0 timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/f_def -o run -- python3 tools/quick_time.py 3,256,10,2")
tools/gpu_steps.sh "${steps[@]}"
