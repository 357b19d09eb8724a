#!/bin/bash
# one GPU call: block order (1 Morton, 2 Hilbert) x store policy (plain, sc1) of the dense tier kernels
cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "120:ord_plain:python -u tools/quick_time.py 3,256,6,1 3,256,6,2 3,256,8,1 3,256,8,2 3,256,6,1" \
  "120:ord_sc1:GM_LIB_PATH=_exp/libgm_sc1.so python -u tools/quick_time.py 3,256,6,1 3,256,6,2 3,256,8,1 3,256,8,2" \
  "120:ord_exp1:GM_LIB_PATH=_exp/libgm_exp1.so python -u tools/quick_time.py 3,256,6,1 3,256,6,2" \
  "120:ord_exp1sc1:GM_LIB_PATH=_exp/libgm_exp1sc1.so python -u tools/quick_time.py 3,256,6,1 3,256,6,2"
