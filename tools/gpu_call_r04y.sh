#!/bin/bash
# expand variants: the table-full flag read every parent or every 32nd; the next parent's
# key loaded before this one's inserts (GM_SP_ERR_EVERY, GM_SP_PREFETCH in sparse.hip)
mkdir -p gpurun_out/r04y_exp
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for v in e1p0 e32p0 e1p1 e32p1 e32p3; do
    GM_LIB_PATH=_exp/libgm_$v.so timeout -k 10 120 python tools/solve_timed.py toot 6 4 6 > gpurun_out/r04y_exp/${v}_$rep.log 2>&1 || exit 1
  done
done
