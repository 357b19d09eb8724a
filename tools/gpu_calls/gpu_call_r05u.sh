#!/bin/bash
# Round 5: the split tier kernel with per-tier fill dispatch (a launch without transposed children
# reads as at N = 1; in-tree) against the round-5 kernel (_exp plain0), solo spans G = 2 / 4 / 8;
# then the split parity tests with the in-tree build.
set -o pipefail
mkdir -p gpurun_out/r05u
for v in default plain0 default2 plain0b; do
  lib=""
  case $v in plain0*) lib=_exp/libgm_plain0.so;; esac
  GM_LIB_PATH=$lib timeout -k 10 300 python -X faulthandler -u tools/box_split_time.py --ranks 2 4 8 --reps 3 --batch 1 \
      > gpurun_out/r05u/$v.txt 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_sharded.py -k "box_split" \
    > gpurun_out/r05u/pytest_split.txt 2>&1 || exit 1
