#!/bin/bash
cd "$GRAFT_REPO_ROOT"
steps=()
for m in 0 1024 2048 4096 8192 16384; do steps+=("60:wkmin_$m:GM_WK_MIN=$m python -u tools/quick_time.py 3,256,10,2 3,256,10,2"); done
tools/gpu_steps.sh "${steps[@]}"
