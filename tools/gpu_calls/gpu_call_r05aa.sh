#!/bin/bash
# Round 5: the walk with the b0 / b1 neighbours from the LDS image (GM_BOX_WALK_B01 1: 2 VALU fewer
# per step, 75 steps instead of 73) against the default, N = 1 kernel ms, three interleaved passes.
set -o pipefail
mkdir -p gpurun_out/r05aa
libs="gamesmanmpi_amd/libgmsolve.so _exp/libgm_b01.so"
timeout -k 10 400 python -u tools/box_variants.py $libs $libs $libs > gpurun_out/r05aa/walk_b01.txt 2>&1 || exit 1
