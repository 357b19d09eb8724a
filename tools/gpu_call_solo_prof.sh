#!/bin/bash
# Kernel traces of one rank's tier launches alone (GM_OPT_DIST_SOLO) against the
# single-GPU solve (graph replay and eager), for the per-rank critical path.
export TMPDIR=/tmp
O=$(pwd)/gpurun_out
tools/gpu_steps.sh \
 "120:eager1:GM_OPT_GRAPH=0 python tools/solve_timed.py subtract 8 6" \
 "180:kt_solo8:GM_OPT_DIST_SOLO=1 rocprofv3 --kernel-trace --output-format csv -d $O/kt_solo8 -o run -- python3 tools/solve_timed.py subtract 8 4 8" \
 "180:kt_single:rocprofv3 --kernel-trace --output-format csv -d $O/kt_single -o run -- python3 tools/solve_timed.py subtract 8 4"
