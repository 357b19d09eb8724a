#!/bin/bash
# Round 5: Toot 6x4 with the locality home of the tier tables (GM_SPARSE_HOME_W), per window size.
set -o pipefail
mkdir -p gpurun_out/r05f
for w in 0 6 10 14 18 0; do
    echo "== GM_SPARSE_HOME_W=$w" >> gpurun_out/r05f/home_sweep.txt
    GM_SPARSE_HOME_W=$w timeout -k 10 240 python -u tools/solve_timed.py toot 6 4 5 >> gpurun_out/r05f/home_sweep.txt 2>&1 || exit 1
done
