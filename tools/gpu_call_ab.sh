set -o pipefail
O=gpurun_out
tools/gpu_steps.sh \
 "600:sharded:python -u -m pytest tests/test_gpu_sharded.py -x -q --timeout 300 --timeout-method thread" \
 "120:old_v8:GM_LIB_PATH=_exp/libgm_old.so python tools/solve_timed.py subtract 8 6 8" \
 "120:new_v8:python tools/solve_timed.py subtract 8 6 8" \
 "120:old_v2:GM_LIB_PATH=_exp/libgm_old.so python tools/solve_timed.py subtract 8 6 2" \
 "120:new_v2:python tools/solve_timed.py subtract 8 6 2" \
 "120:solo8_r0:GM_OPT_DIST_SOLO=1 python tools/solve_timed.py subtract 8 6 8" \
 "120:solo8_r7:GM_OPT_DIST_SOLO=8 python tools/solve_timed.py subtract 8 6 8" \
 "120:solo4_r3:GM_OPT_DIST_SOLO=4 python tools/solve_timed.py subtract 8 6 4" \
 "120:solo2_r1:GM_OPT_DIST_SOLO=2 python tools/solve_timed.py subtract 8 6 2" \
 "300:bench:python bench.py"
