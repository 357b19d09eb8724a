#!/bin/bash
# one GPU call: one-block workgroups for the small head/tail tiers (GM_SMALL_TIER threshold)
cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "100:small0:python -u tools/quick_time.py 3,256,6,2 3,256,6,2" \
  "100:small512:GM_SMALL_TIER=512 python -u tools/quick_time.py 3,256,6,2 3,256,6,2" \
  "100:small1024:GM_SMALL_TIER=1024 python -u tools/quick_time.py 3,256,6,2 3,256,6,2" \
  "100:small2048:GM_SMALL_TIER=2048 python -u tools/quick_time.py 3,256,6,2 3,256,6,2" \
  "100:small4096:GM_SMALL_TIER=4096 python -u tools/quick_time.py 3,256,6,2 3,256,6,2" \
  "100:small8192:GM_SMALL_TIER=8192 python -u tools/quick_time.py 3,256,6,2 3,256,6,2"
tools/gpu_steps.sh \
  "100:pw8:GM_LIB_PATH=_exp/libgm_pw8.so python -u tools/quick_time.py 3,256,6,2 3,256,6,2" \
  "100:pw:GM_LIB_PATH=_exp/libgm_pw.so python -u tools/quick_time.py 3,256,6,2 3,256,6,2" \
  "100:pw8s2048:GM_SMALL_TIER=2048 GM_LIB_PATH=_exp/libgm_pw8.so python -u tools/quick_time.py 3,256,6,2 3,256,6,2"
