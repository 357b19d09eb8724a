#!/bin/bash
# pass-B-only (exp6) and full solve time against workgroups per CU (unused LDS pad)
cd "$GRAFT_REPO_ROOT"
steps=()
steps+=("60:occ_base7:GM_LIB_PATH=_exp/libgm_exp7.so python -u tools/quick_time.py 3,256,10,2 3,256,6,2")
for pad in 0 21504 63232 102400; do
  steps+=("60:occ_wk6_$pad:GM_PAD_LDS=$pad GM_LIB_PATH=_exp/libgm_exp6.so python -u tools/quick_time.py 3,256,10,2")
  steps+=("60:occ_wk_$pad:GM_PAD_LDS=$pad python -u tools/quick_time.py 3,256,10,2")
done
for pad in 0 65536 102400; do
  steps+=("60:occ_b46_$pad:GM_PAD_LDS=$pad GM_LIB_PATH=_exp/libgm_exp6.so python -u tools/quick_time.py 3,256,6,2")
done
tools/gpu_steps.sh "${steps[@]}"
