#!/bin/bash
cd "$GRAFT_REPO_ROOT"
steps=("300:wk_parity:python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k 'variants and (10 or 12 or vs_oracle)'")
steps+=("120:wk_time:python -u tools/quick_time.py 3,256,12,2 3,256,10,2 3,256,12,2")
steps+=("60:wk2_walk:GM_LIB_PATH=_exp/libgm_exp6.so python -u tools/quick_time.py 3,256,12,2")
steps+=("60:wk2_nowalk:GM_LIB_PATH=_exp/libgm_exp1.so python -u tools/quick_time.py 3,256,12,2")
tools/gpu_steps.sh "${steps[@]}"
