#!/bin/bash
# one GPU call: block order 2 (Hilbert) vs 3 (Hilbert runs walked by layers, GM_ORDER_LAYER 0..4):
# solve time and FETCH_SIZE of the 2^32 subtract solve
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
steps=("60:o2:python -u tools/quick_time.py 3,256,10,2 3,256,10,2")
steps+=("90:f_o2:timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/f_o2 -o run -- python3 tools/quick_time.py 3,256,10,2")
for L in 0 1 2 3 4; do
  steps+=("60:o3_$L:GM_ORDER_LAYER=$L python -u tools/quick_time.py 3,256,10,2 3,256,10,3 3,256,10,3")
  steps+=("90:f_o3_$L:GM_ORDER_LAYER=$L timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/f_o3_$L -o run -- python3 tools/quick_time.py 3,256,10,3")
done
tools/gpu_steps.sh "${steps[@]}"
