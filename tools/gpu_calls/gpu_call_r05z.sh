#!/bin/bash
# Round 5: the tier launches' store cache policy (GM_BOX_TIER_STORE_CPOL; sc1 = 16 is the default),
# N = 1 kernel ms of the 2^32 solve, two interleaved passes.
set -o pipefail
mkdir -p gpurun_out/r05z
libs="gamesmanmpi_amd/libgmsolve.so _exp/libgm_scp0.so _exp/libgm_scp2.so _exp/libgm_scp18.so _exp/libgm_scp3.so _exp/libgm_scp17.so"
timeout -k 10 500 python -u tools/box_variants.py $libs $libs > gpurun_out/r05z/store_cpol.txt 2>&1 || exit 1
