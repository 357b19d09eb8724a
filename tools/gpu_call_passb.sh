#!/bin/bash
# one GPU call: pass B variants of the b4 kernel (split registers, s_setprio), sc1 stores, Hilbert order
cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "120:pb_sc1:GM_LIB_PATH=_exp/libgm_sc1.so python -u tools/quick_time.py 3,256,6,2 3,256,6,2" \
  "120:pb_prio1:GM_LIB_PATH=_exp/libgm_prio1.so python -u tools/quick_time.py 3,256,6,2 3,256,6,2" \
  "120:pb_prio3:GM_LIB_PATH=_exp/libgm_prio3.so python -u tools/quick_time.py 3,256,6,2 3,256,6,2" \
  "120:pb_split:GM_LIB_PATH=_exp/libgm_split.so python -u tools/quick_time.py 3,256,6,2 3,256,6,2" \
  "120:pb_splitprio1:GM_LIB_PATH=_exp/libgm_splitprio1.so python -u tools/quick_time.py 3,256,6,2 3,256,6,2"
