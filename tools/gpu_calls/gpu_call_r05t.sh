#!/bin/bash
# Round 5: the split tier kernel's fill-free groups issuing their loads as at N = 1
# (GM_BOX_SPLIT_PLAIN 1, in-tree) against the round's kernel (0), solo spans G = 2 / 4 / 8;
# then the split parity tests with the in-tree build.
set -o pipefail
mkdir -p gpurun_out/r05t
for v in default plain0 default2; do
  lib=""
  [ "$v" = plain0 ] && lib=_exp/libgm_$v.so
  GM_LIB_PATH=$lib timeout -k 10 300 python -X faulthandler -u tools/box_split_time.py --ranks 2 4 8 --reps 3 --batch 1 \
      > gpurun_out/r05t/$v.txt 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_sharded.py -k "box_split" \
    > gpurun_out/r05t/pytest_split.txt 2>&1 || exit 1
