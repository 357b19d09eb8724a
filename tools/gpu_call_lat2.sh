#!/bin/bash
# one GPU call: latency variant as the default tier kernel vs the load-barrier build (168 VGPRs)
cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "100:def:python -u tools/quick_time.py 3,256,6,2 3,256,6,2 3,256,6,2" \
  "100:latbar:GM_LIB_PATH=_exp/libgm_latbar.so python -u tools/quick_time.py 3,256,6,2 3,256,6,2 3,256,6,2" \
  "300:solo_latbar:GM_LIB_PATH=_exp/libgm_latbar.so python -u tools/solo_variants.py 8"
