#!/bin/bash
# walker kernel (GM_OPT_SUB_INTERLEAVE 10): parity, timing against b4, ablation
cd "$GRAFT_REPO_ROOT"
steps=("300:wk_parity:python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k 'variants and (10 or vs_oracle)'")
steps+=("120:wk_time:python -u tools/quick_time.py 3,256,6,2 3,256,10,2 3,256,10,1")
steps+=("120:wk_time_w1:GM_LIB_PATH=_exp/libgm_wk1.so python -u tools/quick_time.py 3,256,10,2")
for n in 1 2 4 5 6; do steps+=("120:wk_abl$n:GM_LIB_PATH=_exp/libgm_exp$n.so python -u tools/quick_time.py 3,256,10,2"); done
steps+=("150:wk_kt:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wk_kt -o run -- python3 -u tools/quick_time.py 3,256,10,2")
tools/gpu_steps.sh "${steps[@]}"
