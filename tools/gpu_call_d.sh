tools/gpu_steps.sh \
  "300:abl0:python tools/quick_time.py 3,256,4,1" \
  "300:abl1:GM_LIB_PATH=_exp/libgm_exp1.so python tools/quick_time.py 3,256,4,1" \
  "300:abl2:GM_LIB_PATH=_exp/libgm_exp2.so python tools/quick_time.py 3,256,4,1" \
  "300:abl3:GM_LIB_PATH=_exp/libgm_exp3.so python tools/quick_time.py 3,256,4,1" \
  "120:pmc_l2:timeout -s KILL 100 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_l2 -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline" \
  "60:listavail:rocprofv3 --list-avail > gpurun_out/list_avail.txt 2>&1 || true" \
  "150:toot_trace:GM_TRACE=1 python -u tools/solve_timed.py toot 6 4 2"
