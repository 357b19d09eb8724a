#!/bin/bash
cd "$GRAFT_REPO_ROOT"
steps=("300:parity:python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k 'variants or walker or subtract'")
steps+=("60:skip:python -u tools/quick_time.py 3,256,10,2 3,256,10,2 3,256,6,2")
steps+=("60:noskip:GM_LIB_PATH=_exp/libgm_noskip.so python -u tools/quick_time.py 3,256,10,2 3,256,10,2 3,256,6,2")
steps+=("60:loads_skip:GM_LIB_PATH=_exp/libgm_exp5.so python -u tools/quick_time.py 3,256,10,2")
steps+=("60:loads_noskip:GM_LIB_PATH=_exp/libgm_e5noskip.so python -u tools/quick_time.py 3,256,10,2")
steps+=("90:fetch:timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/skip_fetch -o run -- python3 tools/quick_time.py 3,256,10,2")
tools/gpu_steps.sh "${steps[@]}"
