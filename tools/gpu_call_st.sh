#!/bin/bash
cd "$GRAFT_REPO_ROOT"
steps=("120:st_def:python -u tools/quick_time.py 3,256,10,2")
for t in st0 st2 st18 st3 st17; do steps+=("60:$t:GM_LIB_PATH=_exp/libgm_$t.so python -u tools/quick_time.py 3,256,10,2"); done
tools/gpu_steps.sh "${steps[@]}"
