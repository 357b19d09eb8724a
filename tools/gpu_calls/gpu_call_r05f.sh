#!/bin/bash
# Round 5: Toot 6x4 with the locality home of the tier tables (GM_SPARSE_HOME_W), per window size.
# A window too small for a group overflows the table: a clean error (exit 1), the sweep goes on;
# any other failure ends it.
set -o pipefail
mkdir -p gpurun_out/r05f
for w in 12 16 20 24 0; do
    echo "== GM_SPARSE_HOME_W=$w" >> gpurun_out/r05f/home_sweep2.txt
    GM_SPARSE_HOME_W=$w timeout -k 10 240 python -u tools/solve_timed.py toot 6 4 5 >> gpurun_out/r05f/home_sweep2.txt 2>&1
    rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
