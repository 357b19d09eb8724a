#!/bin/bash
# Round 5: where a split rank's extra time per box goes -- the split tier kernel as built, with
# children read as at N = 1 (GM_BOX_EXP 16: exact for rank 0, which has no fills), and also
# without the halo stores (48).  Solo spans per rank, G = 2 / 4 / 8.
set -o pipefail
mkdir -p gpurun_out/r05s
for v in default exp16 exp48; do
  lib=""
  [ "$v" != default ] && lib=_exp/libgm_$v.so
  GM_LIB_PATH=$lib timeout -k 10 400 python -X faulthandler -u tools/box_split_time.py --ranks 2 4 8 --reps 3 --batch 1 \
      > gpurun_out/r05s/$v.txt 2>&1 || exit 1
done
