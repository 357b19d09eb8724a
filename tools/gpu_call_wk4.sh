#!/bin/bash
cd "$GRAFT_REPO_ROOT"
steps=("300:wk_parity:python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k 'variants and (10 or vs_oracle)'")
steps+=("120:wk_time:python -u tools/quick_time.py 3,256,10,2 3,256,6,2")
steps+=("60:wk_nt256:GM_LIB_PATH=_exp/libgm_nt256.so python -u tools/quick_time.py 3,256,10,2")
steps+=("60:wk_walk:GM_LIB_PATH=_exp/libgm_exp6.so python -u tools/quick_time.py 3,256,10,2")
steps+=("60:wk_base:GM_LIB_PATH=_exp/libgm_exp7.so python -u tools/quick_time.py 3,256,10,2")
steps+=("120:trace:GM_LIB_PATH=_exp/libgm_tr.so python -u tools/wk_trace.py")
tools/gpu_steps.sh "${steps[@]}"
