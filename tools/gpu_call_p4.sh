#!/bin/bash
# one GPU call: the pipelined persistent dense kernel (GM_OPT_SUB_INTERLEAVE 9): parity, timing, kernel trace
cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "300:p4_tests:python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k 'variants'" \
  "120:p4_time:python -u tools/quick_time.py 3,256,6,2 3,256,9,2 3,256,9,1 3,256,6,2 3,256,9,2" \
  "120:p4_w5:GM_LIB_PATH=_exp/libgm_p4w5.so python -u tools/quick_time.py 3,256,9,2 3,256,9,2" \
  "120:p4_sc1:GM_LIB_PATH=_exp/libgm_p4sc1.so python -u tools/quick_time.py 3,256,9,2 3,256,9,2" \
  "150:p4_kt:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p4_kt -- python3 -u tools/quick_time.py 3,256,9,2"
