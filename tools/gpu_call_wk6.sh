#!/bin/bash
cd "$GRAFT_REPO_ROOT"
steps=()
for p in 1 2 3; do
steps+=("60:wk_p$p:GM_WKP_PER_CU=$p python -u tools/quick_time.py 3,256,11,2")
steps+=("60:wk_nowalk_p$p:GM_WKP_PER_CU=$p GM_LIB_PATH=_exp/libgm_exp1.so python -u tools/quick_time.py 3,256,11,2")
steps+=("60:wk_walk_p$p:GM_WKP_PER_CU=$p GM_LIB_PATH=_exp/libgm_exp6.so python -u tools/quick_time.py 3,256,11,2")
done
tools/gpu_steps.sh "${steps[@]}"
