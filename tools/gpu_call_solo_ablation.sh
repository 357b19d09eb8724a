#!/bin/bash
# Phase ablation of one rank's tier launches at G = 8 (GM_OPT_DIST_SOLO=1): kernel
# traces of the full kernel and of builds without pass B (exp1), without child loads
# (exp2) and without both (exp3); tools/build_exp.sh makes the _exp libraries.
export TMPDIR=/tmp
O=$(pwd)/gpurun_out
steps=()
for v in base exp1 exp2 exp3; do
  lib=""; [ $v != base ] && lib="GM_LIB_PATH=_exp/libgm_$v.so"
  steps+=("180:abl_$v:$lib GM_OPT_DIST_SOLO=1 rocprofv3 --kernel-trace --output-format csv -d $O/abl_$v -o run -- python3 tools/solve_timed.py subtract 8 4 8")
done
steps+=("180:abl_single_exp1:GM_LIB_PATH=_exp/libgm_exp1.so rocprofv3 --kernel-trace --output-format csv -d $O/abl_single_exp1 -o run -- python3 tools/solve_timed.py subtract 8 4")
tools/gpu_steps.sh "${steps[@]}"
