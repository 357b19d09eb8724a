#!/bin/bash
# one GPU call: the one-wave dense kernel (GM_OPT_SUB_INTERLEAVE 8) -- parity tests of the
# kernel variants, then timing against the b4 kernel and a kernel trace of both
cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "300:w1_tests:python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k 'variants or full_table_vs_oracle or 7_heaps'" \
  "120:w1_time:python -u tools/quick_time.py 3,256,6 3,256,8 3,256,6 3,256,8" \
  "150:w1_kt:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/w1_kt -- python3 -u tools/quick_time.py 3,256,8 3,256,6"
