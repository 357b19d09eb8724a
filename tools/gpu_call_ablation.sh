#!/bin/bash
# dense kernel phase ablation: 1 no pass B, 2 no child loads, 4 no stores (bits combine)
cd "$GRAFT_REPO_ROOT"
steps=("120:abl0:python -u tools/quick_time.py 3,256,6")
for n in 1 2 3 4 5 6 7; do steps+=("120:abl$n:GM_LIB_PATH=_exp/libgm_exp$n.so python -u tools/quick_time.py 3,256,6"); done
steps+=("150:kt_full:rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_full -- python3 -u tools/quick_time.py 3,256,6")
tools/gpu_steps.sh "${steps[@]}"
