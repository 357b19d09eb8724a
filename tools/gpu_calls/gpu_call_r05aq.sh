#!/bin/bash
# Round 5: LLVM AMDGPU scheduler strategies on dense_box.hip (max-ilp, metric bias 0,
# max-memory-clause) against the default, N = 1 kernel ms, two interleaved passes.
set -o pipefail
mkdir -p gpurun_out/r05aq
libs="gamesmanmpi_amd/libgmsolve.so _exp/libgm_ilp.so _exp/libgm_bias0.so _exp/libgm_lat.so"
timeout -k 10 500 python -u tools/box_variants.py $libs $libs > gpurun_out/r05aq/sched.txt 2>&1 || exit 1
